#!/usr/bin/env python3
"""Products-phase time against k at a fixed m = n (fast mode, N = 14): python products_k.py <m> <k> [<k> ...].
Run it with GEMMUL8_PERSISTENT=0 / 1 to compare the one-tile and the persistent kernel per k-step count."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
import gemmul8 as G  # noqa: E402


def main():
    m = n = int(sys.argv[1])
    N = 14
    for k in (int(x) for x in sys.argv[2:]):
        A = G.randmat(m, k, torch.float64, 0.5, 123456)
        B = G.randmat(k, n, torch.float64, 0.5, 654321)
        C = torch.empty((n, m), dtype=torch.float64, device="cuda")
        w = G.alloc_work(m, n, k, N)
        call = lambda: G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, True, w, phase_times=True)
        for _ in range(5):
            call()
        ph = [0.0] * 4
        for _ in range(30):
            ph = [a + b / 30e3 for a, b in zip(ph, call())]
        print(json.dumps({"m": m, "k": k, "ksteps": (k + 63) // 64, "kernel": G.last_products_kernel(),
                          "phases_us": [round(x, 2) for x in ph]}), flush=True)
        del A, B, C, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
