#!/usr/bin/env python3
"""Profiling target: a few cfg2 calls (DGEMM emulation 8192^3, 14 moduli, fast) through the C ABI."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
import gemmul8 as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=8192)
ap.add_argument("--moduli", type=int, default=14)
ap.add_argument("--calls", type=int, default=3)
ap.add_argument("--accurate", action="store_true")
a = ap.parse_args()
m = n = k = a.size
A = G.randmat(m, k, torch.float64, 0.5, 123456)
B = G.randmat(k, n, torch.float64, 0.5, 123456)
C = torch.empty((n, m), dtype=torch.float64, device="cuda")
W = G.alloc_work(m, n, k, a.moduli)
for _ in range(a.calls):
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, a.moduli, not a.accurate, W)
torch.cuda.synchronize()
print("done")
