"""Integer inputs: the emulation against the CPU oracle (bits) and the exact product (error size)."""
import sys, numpy as np, torch
sys.path[:0] = ["tests", ".", "mixed-gemmul8_amd"]
import gemmul8 as G
from oracle import oracle as O
from test_gpu_parity import run_gpu
rng = np.random.default_rng(3)
for (m, n, k) in [(512, 384, 1536), (300, 200, 64)]:
    A = np.asfortranarray(rng.integers(-1000, 1001, (m, k)).astype(np.float64))
    B = np.asfortranarray(rng.integers(-1000, 1001, (k, n)).astype(np.float64))
    ex = A @ B
    for fast in (True, False):
        C, _, _ = run_gpu(A, B, 14, fast=fast)
        Co = O.gemm(A, B, 14, fast)
        d = np.abs(C - ex)
        print(m, n, k, "fast" if fast else "accu", "gpu==oracle", np.asfortranarray(C).tobytes() == np.asfortranarray(Co).tobytes(),
              "mismatch vs exact", int((d > 0).sum()), "max abs", float(d.max()), "max rel", float((d / np.maximum(np.abs(ex), 1)).max()))
