#!/usr/bin/env python3
"""Profiling target: a few emulated GEMM calls through the C ABI.

--cfg 2 (default): DGEMM 8192^3 (or --size), 14 moduli, fast mode;
--cfg 4: A f64 x B f32 -> C f64, 8192^3, 10 moduli, accurate mode (BASELINE.json configs[3]);
--cfg 5: complex f64 4096^3, 12 moduli, COMPLEX_BIG_MATRIX_ENCODE, fast mode (configs[4]).
--reads: afterwards, calibration reads of known bytes (torch.sum, 3 each) over a 4 GiB tensor (from HBM:
beyond the 256 MiB Infinity Cache) and a 128 MiB one (beyond the 32 MiB of L2, inside the Infinity Cache),
to tell what a memory-side counter sees of each.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
import gemmul8 as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", type=int, default=2, choices=[2, 4, 5])
ap.add_argument("--size", type=int, default=0)
ap.add_argument("--moduli", type=int, default=0)
ap.add_argument("--calls", type=int, default=3)
ap.add_argument("--accurate", action="store_true")
ap.add_argument("--reads", action="store_true")
a = ap.parse_args()
ta, tb, tc, N, fast, ctype, size = torch.float64, torch.float64, torch.float64, 14, not a.accurate, G.REAL_DEFAULT, 8192
if a.cfg == 4:
    tb, N, fast = torch.float32, 10, False
elif a.cfg == 5:
    ta = tb = tc = torch.complex128
    N, ctype, size = 12, G.COMPLEX_BIG_MATRIX_ENCODE, 4096
m = n = k = a.size or size
N = a.moduli or N
A = G.randmat(m, k, ta, 0.5, 123456)
B = G.randmat(k, n, tb, 0.5, 123456)
C = torch.empty((n, m), dtype=tc, device="cuda")
W = G.alloc_work(m, n, k, N, ctype)
for _ in range(a.calls):
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, W, ctype)
torch.cuda.synchronize()
if a.reads:
    del A, B, C, W
    torch.cuda.empty_cache()
    for elems in (512 << 20, 16 << 20):  # 4 GiB, 128 MiB of float64
        X = torch.ones(elems, dtype=torch.float64, device="cuda")
        for _ in range(3):
            X.sum()
        torch.cuda.synchronize()
        del X
print("done")
