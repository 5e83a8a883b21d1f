#!/usr/bin/env python3
"""Product-phase time against k at a fixed m = n (one round of tiles or a few): the intercept is the
per-launch fixed cost of the residue product kernel, the slope its time per k-step."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
import gemmul8 as G  # noqa: E402

mn = [int(x) for x in (sys.argv[1:] or ["1024", "2048"])]
for s in mn:
    for k in (64, 128, 256, 384, 512, 1024, 2048, 4096):
        m = n = s
        A = G.randmat(m, k, torch.float64, 0.5, 123456)
        B = G.randmat(k, n, torch.float64, 0.5, 654321)
        C = torch.empty((n, m), dtype=torch.float64, device="cuda")
        W = G.alloc_work(m, n, k, 14)
        for _ in range(5):
            G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, True, W)
        G.timing_enable(True)
        G.timing_read()
        for _ in range(50):
            G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, True, W)
        G.timing_enable(False)
        ph, calls = G.timing_read()
        print(f"m=n={s} k={k:5d} ksteps={k // 64:3d}: split {ph[0] / calls * 1e3:7.1f} us, products "
              f"{ph[1] / calls * 1e3:7.1f} us, crt {ph[3] / calls * 1e3:6.1f} us", flush=True)
