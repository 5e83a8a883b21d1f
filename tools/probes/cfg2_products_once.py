#!/usr/bin/env python3
"""cfg2's call (8192^3, N = 14, fast) a few times, for counter passes over the product kernel of a given build:
python cfg2_products_once.py [calls]; GEMMUL8_PKG=<dir holding gemmul8/> picks the build."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.environ.get("GEMMUL8_PKG") or os.path.join(ROOT, "mixed-gemmul8_amd"))
import gemmul8 as G  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 3
m = 8192
A = G.randmat(m, m, torch.float64, 0.5, 123456)
C = torch.empty((m, m), dtype=torch.float64, device="cuda")
w = G.alloc_work(m, m, m, 14)
for _ in range(calls):
    G.gemm(G.OP_N, G.OP_N, m, m, m, 1.0, A, m, A, m, 0.0, C, m, 14, True, w)
torch.cuda.synchronize()
print("done", G.last_products_kernel())
