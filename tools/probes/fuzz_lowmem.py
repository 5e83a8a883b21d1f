#!/usr/bin/env python3
"""Randomised check of the low-memory mode (gemmul8_gemm_lowmem: slice_planes S < N, the moduli
encoded and multiplied in groups of S through the same planes) against the resident call: random
shapes, N, S, types, fast/accurate, ops, complex compute types; C must be the same bits.
python fuzz_lowmem.py [cases] [seed]"""
import sys
import time

import numpy as np
import torch

sys.path[:0] = ["tests", ".", "mixed-gemmul8_amd"]
import gemmul8 as G  # noqa: E402

TYPES = {"d": torch.float64, "s": torch.float32, "z": torch.complex128, "c": torch.complex64}
COMBOS = ["ddd", "sss", "dsd", "sdd", "dss", "sds", "ccc", "zzz", "czz", "zcz", "zcc", "czc"]
cases = int(sys.argv[1]) if len(sys.argv) > 1 else 200
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
t0 = time.time()
fails = 0
for c in range(cases):
    ta, tb, tc = COMBOS[rng.integers(len(COMBOS))]
    cplx = ta in "cz"
    m, n, k = (int(rng.integers(1, 700)) for _ in range(3))
    N = int(rng.integers(3, 21))
    S = int(rng.integers(1, N))
    fast = bool(rng.integers(2))
    opA, opB = int(rng.integers(3 if cplx else 2)), int(rng.integers(3 if cplx else 2))
    ct = int(rng.integers(1, 4)) if cplx else 0
    g = torch.Generator(device="cuda").manual_seed(c)

    def mat(r, q, t):
        dt = TYPES[t]
        if dt.is_complex:
            re = torch.float64 if dt == torch.complex128 else torch.float32
            return torch.complex(torch.randn(q, r, dtype=re, device="cuda", generator=g),
                                 torch.randn(q, r, dtype=re, device="cuda", generator=g))
        return torch.randn(q, r, dtype=dt, device="cuda", generator=g)

    A = mat(k, m, ta) if opA else mat(m, k, ta)   # column-major (rows x cols) as (cols, rows) row-major
    B = mat(n, k, tb) if opB else mat(k, n, tb)
    lda, ldb = (k if opA else m), (n if opB else k)
    out = []
    for sp in (None, S):
        C = torch.zeros((n, m), dtype=TYPES[tc], device="cuda")
        W = G.alloc_work(m, n, k, N, ct, slice_planes=sp)
        G.gemm(opA, opB, m, n, k, 1.0, A, lda, B, ldb, 0.0, C, m, N, fast, W, ct, slice_planes=sp)
        out.append(C)
    torch.cuda.synchronize()
    bits = [torch.view_as_real(x) if cplx else x for x in out]
    same = torch.equal(bits[0].contiguous().view(torch.uint8), bits[1].contiguous().view(torch.uint8))
    if not same:
        fails += 1
        print(f"FAIL {ta}{tb}{tc} m={m} n={n} k={k} N={N} S={S} {'fast' if fast else 'accu'} op={opA}{opB} ct={ct}",
              flush=True)
    if (c + 1) % 50 == 0:
        print(f"{c + 1} cases, {fails} failures, {time.time() - t0:.0f} s", flush=True)
print(f"{cases} cases, {fails} failures, {time.time() - t0:.0f} s")
