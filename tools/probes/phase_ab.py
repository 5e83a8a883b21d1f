#!/usr/bin/env python3
"""Phase times (library HIP events) of a gemmul8 package directory: python phase_ab.py PKGDIR [cfg]
cfg 2: DGEMM 8192^3 N=14 fast; 5: complex 4096^3 N=12 big-matrix.  For same-box A/B of two builds
(copy a built package to another directory and run both)."""
import sys

import torch

sys.path.insert(0, sys.argv[1])
import gemmul8 as G  # noqa: E402

cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
if cfg == 5:
    dt, m, N, ct = torch.complex128, 4096, 12, G.COMPLEX_BIG_MATRIX_ENCODE
else:
    dt, m, N, ct = torch.float64, 8192, 14, G.REAL_DEFAULT
A = G.randmat(m, m, dt, 0.5, 123456)
B = G.randmat(m, m, dt, 0.5, 123456)
C = torch.empty((m, m), dtype=dt, device="cuda")
W = G.alloc_work(m, m, m, N, ct)
for _ in range(3):
    G.gemm(0, 0, m, m, m, 1.0, A, m, B, m, 0.0, C, m, N, True, W, ct)
G.timing_enable(True)
G.timing_read()
for _ in range(20):
    G.gemm(0, 0, m, m, m, 1.0, A, m, B, m, 0.0, C, m, N, True, W, ct)
torch.cuda.synchronize()
G.timing_enable(False)
ms, calls = G.timing_read()
print(sys.argv[1], "cfg", cfg, " ".join(f"{x / calls:.4f}" for x in ms), "ms (split, products, -, crt)")
