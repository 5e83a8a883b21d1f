"""dist_soak.py -- test infrastructure: random cases of gemmul8.dist's NCCL branch through tests/fake_nccl.py
(ranks as threads on one GPU): shapes, moduli counts, rank counts 2..5, fast / accurate, real / complex (with
Karatsuba products), unit orders, side stream on / off, C gathered or distributed, random transfer delays, two
calls per case through the same workspaces.  Every rank's output is compared bit for bit with the single
gemmul8_gemm call.  Used by tests/test_gpu_dist_streams.py (a short run); long soaks: python tests/dist_soak.py [cases] [seed]."""
import os

import numpy as np
import torch

from fake_nccl import FakeNcclWorld, run_ranks
from test_gpu_phases import _rand, _same, _single


def random_case(rng):
    W = int(rng.integers(2, 6))
    cplx = bool(rng.random() < 0.25)
    fast = bool(rng.random() < 0.7)
    N = int(rng.integers(2, 20 if cplx else 21))
    m = int(rng.integers(1, 1300))
    n = int(rng.integers(1, 257 * W + 600))
    k = int(rng.integers(1, 1500)) if not cplx or rng.random() < 0.7 else int(rng.integers(3072, 3300))
    if cplx and k >= 3072:
        m = max(m, 1024)  # the Karatsuba product form (three residue sub-planes per transfer)
    return dict(W=W, cplx=cplx, fast=fast, N=N, m=m, n=n, k=k,
                order="columns" if rng.random() < 0.3 else "moduli", gather=bool(rng.random() < 0.4),
                side=bool(rng.random() < 0.7), delay=int(rng.choice([0, 50_000, 400_000])),
                seeds=[int(x) for x in rng.integers(1000, 10 ** 6, size=2)])


def run_case(c):
    """None when every rank's output equals the single call's, else a description of the first difference"""
    from gemmul8 import dist as GD
    W, N, m, n, k, fast = c["W"], c["N"], c["m"], c["n"], c["k"], c["fast"]
    dt = torch.complex128 if c["cplx"] else torch.float64
    data = [(_rand(m, k, s, dt), _rand(k, n, s + 1, dt)) for s in c["seeds"]]
    torch.cuda.synchronize()
    refs = [_single(A, B, N, fast, dt) for A, B in data]
    plan = GD.ShardPlan(m, n, N, W, order=c["order"])
    world = FakeNcclWorld(W, delay_cycles=c["delay"])
    real_dist, env = GD.dist, os.environ.get("GEMMUL8_DIST_SIDE_STREAM")
    GD.dist = world.module
    os.environ["GEMMUL8_DIST_SIDE_STREAM"] = "1" if c["side"] else "0"

    def rank(r):
        ops = GD.HipShardOps()
        comp = torch.cuda.Stream()
        with torch.cuda.stream(comp):
            out = [GD.matmul_moduli(A, B, N, fast, gather=c["gather"], ops=ops, order=c["order"]) for A, B in data]
        comp.synchronize()
        return out

    try:
        res = run_ranks(world, rank)
    finally:
        GD.dist = real_dist
        if env is None:
            os.environ.pop("GEMMUL8_DIST_SIDE_STREAM", None)
        else:
            os.environ["GEMMUL8_DIST_SIDE_STREAM"] = env
    for i, ref in enumerate(refs):
        for r in range(W):
            if c["gather"]:
                ok = _same(res[r][i], ref) if r == 0 else res[r][i] is None
            else:
                c0, c1 = plan.cols[r]
                ok = (c1 == c0 and res[r][i].numel() == 0) or _same(res[r][i], ref[:, c0:c1])
            if not ok:
                return f"call {i} rank {r} differs"
    return None


def soak(cases, seed, log=None):
    """(number of failures, [(case, message)]) over `cases` random cases"""
    rng = np.random.default_rng(seed)
    fails = []
    for i in range(cases):
        c = random_case(rng)
        try:
            msg = run_case(c)
        except Exception as e:  # report and go on
            msg = f"{type(e).__name__}: {str(e)[:200]}"
        if msg:
            fails.append((c, msg))
        if log and (i + 1) % 10 == 0:
            log(f"{i + 1} cases, {len(fails)} failures")
    return len(fails), fails


if __name__ == "__main__":
    import sys
    import time
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    t0 = time.time()
    n, fails = soak(cases, seed, log=lambda s: print(f"{s}, {time.time() - t0:.0f} s", flush=True))
    for c, msg in fails:
        print("FAIL", c, msg, flush=True)
    print(f"done: {cases} cases, {n} failures, {time.time() - t0:.0f} s")
    sys.exit(1 if n else 0)
