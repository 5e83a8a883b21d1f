#!/usr/bin/env python3
"""Per-call time of 8192^3 N=14 fast emulation for each (opA, opB) on the same operands
(library phase timers)."""
import sys

import torch

sys.path.insert(0, sys.argv[1] if len(sys.argv) > 1 else "mixed-gemmul8_amd")
import gemmul8 as G  # noqa: E402

m = 8192
A = G.randmat(m, m, torch.float64, 0.5, 123456)
B = G.randmat(m, m, torch.float64, 0.5, 654321)
C = torch.empty((m, m), dtype=torch.float64, device="cuda")
W = G.alloc_work(m, m, m, 14)
for opa, opb in ((0, 0), (1, 0), (0, 1), (1, 1)):
    for _ in range(2):
        G.gemm(opa, opb, m, m, m, 1.0, A, m, B, m, 0.0, C, m, 14, True, W)
    G.timing_enable(True)
    G.timing_read()
    for _ in range(10):
        G.gemm(opa, opb, m, m, m, 1.0, A, m, B, m, 0.0, C, m, 14, True, W)
    torch.cuda.synchronize()
    G.timing_enable(False)
    ms, calls = G.timing_read()
    print(f"op({opa},{opb}):", " ".join(f"{x / calls:.4f}" for x in ms), "ms (split, products, -, crt)")
