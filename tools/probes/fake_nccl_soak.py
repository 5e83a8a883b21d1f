#!/usr/bin/env python3
"""Randomised soak of gemmul8.dist's NCCL branch through tests/fake_nccl.py (ranks as threads on one GPU, every
received copy delayed by a GPU spin): random shapes, moduli counts, rank counts 2..5, fast / accurate, real /
complex, unit orders, side stream on / off, C gathered or distributed, two calls per case through the same
workspaces (the second with other operands).  Every rank's output is compared bit for bit with the single
gemmul8_gemm call.  python tools/probes/fake_nccl_soak.py [cases] [seed]"""
import os
import sys
import time

import numpy as np
import torch

sys.path[:0] = ["tests", ".", "mixed-gemmul8_amd"]
from fake_nccl import FakeNcclWorld, run_ranks  # noqa: E402
from test_gpu_phases import _rand, _same, _single  # noqa: E402
from gemmul8 import dist as GD  # noqa: E402

cases = int(sys.argv[1]) if len(sys.argv) > 1 else 50
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
real_dist = GD.dist
t0 = time.time()
fails = 0
for c in range(cases):
    W = int(rng.integers(2, 6))
    cplx = rng.random() < 0.25
    fast = rng.random() < 0.7
    N = int(rng.integers(2, 20 if cplx else 21))
    m = int(rng.integers(1, 1300))
    n = int(rng.integers(1, 257 * W + 600))
    k = int(rng.integers(1, 1500)) if not cplx or rng.random() < 0.7 else int(rng.integers(3072, 3300))
    if cplx and k >= 3072:
        m = max(m, 1024)  # the Karatsuba product form (three residue sub-planes per transfer)
    order = "columns" if rng.random() < 0.3 else "moduli"
    gather = rng.random() < 0.4
    side = rng.random() < 0.7
    dt = torch.complex128 if cplx else torch.float64
    seeds = [int(x) for x in rng.integers(1000, 10 ** 6, size=2)]
    data = [(_rand(m, k, s, dt), _rand(k, n, s + 1, dt)) for s in seeds]
    torch.cuda.synchronize()
    refs = [_single(A, B, N, fast, dt) for A, B in data]
    plan = GD.ShardPlan(m, n, N, W, order=order)
    desc = (f"W={W} {'z' if cplx else 'd'} m={m} n={n} k={k} N={N} {'fast' if fast else 'accu'} order={order} "
            f"gather={gather} side={side}")
    os.environ["GEMMUL8_DIST_SIDE_STREAM"] = "1" if side else "0"
    world = FakeNcclWorld(W, delay_cycles=int(rng.choice([0, 50_000, 400_000])))
    GD.dist = world.module

    def rank(r):
        ops = GD.HipShardOps()
        comp = torch.cuda.Stream()
        with torch.cuda.stream(comp):
            out = [GD.matmul_moduli(A, B, N, fast, gather=gather, ops=ops, order=order) for A, B in data]
        comp.synchronize()
        return out

    try:
        res = run_ranks(world, rank)
        for i, ref in enumerate(refs):
            for r in range(W):
                if gather:
                    ok = _same(res[r][i], ref) if r == 0 else res[r][i] is None
                else:
                    c0, c1 = plan.cols[r]
                    ok = (c1 == c0 and res[r][i].numel() == 0) or _same(res[r][i], ref[:, c0:c1])
                if not ok:
                    raise AssertionError(f"call {i} rank {r} differs")
    except Exception as e:  # report and go on
        fails += 1
        print("FAIL", desc, f"{type(e).__name__}: {str(e)[:200]}", flush=True)
    finally:
        GD.dist = real_dist
    if (c + 1) % 10 == 0:
        print(f"{c + 1} cases, {fails} failures, {time.time() - t0:.0f} s", flush=True)
print(f"done: {cases} cases, {fails} failures, {time.time() - t0:.0f} s")
sys.exit(1 if fails else 0)
