"""Split-phase time at 8192^3 (N = 14, fast) with the default build or the non-temporal-load probe build
(tools/probes/_<name>/gemmul8, e.g. a CRT build with -DOZ2_CRT_NT).  python nt_probe.py default|<name> [reps] [size]"""
import hashlib, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
which = sys.argv[1]
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd") if which == "default" else os.path.join(ROOT, "tools/probes", "_" + which))
import torch
import gemmul8 as G
print(which, G.LIB_PATH, flush=True)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
m = n = k = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
A = G.randmat(m, k, torch.float64, 0.5, 123456)
B = G.randmat(k, n, torch.float64, 0.5, 123456)
C = torch.zeros((n, m), dtype=torch.float64, device="cuda")
W = G.alloc_work(m, n, k, 14)
for _ in range(3):
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, True, W)
torch.cuda.synchronize()
G.timing_enable(True)
G.timing_read()
for _ in range(reps):
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, True, W)
G.timing_enable(False)
ph, calls = G.timing_read()
print(which, m, "ms per call: split %.4f products %.4f crt %.4f" % tuple(x / calls for x in (ph[0], ph[1], ph[3])),
      "C sha1", hashlib.sha1(C.cpu().numpy().tobytes()).hexdigest()[:16], flush=True)
