"""cfg4 shape for rocprofv3 kernel traces: A f64 x B f32 -> C f64, accurate mode, a few calls.
   python mixed_once.py m n k N [iters]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                                "mixed-gemmul8_amd"))
import torch  # noqa: E402
import gemmul8 as G  # noqa: E402

m, n, k, N = (int(x) for x in sys.argv[1:5])
it = int(sys.argv[5]) if len(sys.argv) > 5 else 10
A = torch.randn((k, m), dtype=torch.float64, device="cuda")
B = torch.randn((n, k), dtype=torch.float32, device="cuda")
C = torch.empty((n, m), dtype=torch.float64, device="cuda")
W = G.alloc_work(m, n, k, N)
for _ in range(it):
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, False, W)
torch.cuda.synchronize()
