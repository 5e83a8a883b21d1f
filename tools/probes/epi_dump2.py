"""Like epi_dump.py for one live-fuzz case (probe): v (alpha = 1, beta = 0), C0 and both libraries' C
for the case's alpha / beta.  python epi_dump2.py types m n k N fast ct opA opB alpha beta phi seed"""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mixed-gemmul8_amd"), os.path.dirname(__file__)]
import gemmul8 as G
from test_ref_parity import _ref, CODES
import fuzz_ref as F

ty, m, n, k, N, fast, ct, opA, opB, al, be, phi, seed = sys.argv[1:14]
ta, tb, tc = ty
m, n, k, N, fast, ct, opA, opB, seed = map(int, (m, n, k, N, fast, ct, opA, opB, seed))
al, be, phi = complex(al), complex(be), float(phi)
lib = _ref()
A = G.randmat(k, m, F.TDT[ta], phi, seed) if opA else G.randmat(m, k, F.TDT[ta], phi, seed)
B = G.randmat(n, k, F.TDT[tb], phi, seed + 1) if opB else G.randmat(k, n, F.TDT[tb], phi, seed + 1)
C0 = G.randmat(m, n, F.TDT[tc], 0.5, seed + 2)
lda, ldb = (k if opA else m), (n if opB else k)
out = {}
for name, a, b in (("v", 1, 0), ("x", al, be)):
    Cr, Cn = C0.clone(), C0.clone()
    alpha, beta = np.array([a], F.NPT[tc]), np.array([b], F.NPT[tc])
    w = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + 16 * max(A.numel(), B.numel()) + (1 << 22), dtype=torch.uint8, device="cuda")
    lib.ref_gemm(CODES[ta], CODES[tb], CODES[tc], opA, opB, m, n, k, alpha.ctypes.data, A.data_ptr(), lda, B.data_ptr(), ldb,
                 beta.ctypes.data, Cr.data_ptr(), m, N, fast, ct, w.data_ptr(), None)
    G.gemm(opA, opB, m, n, k, complex(a), A, lda, B, ldb, complex(b), Cn, m, N, bool(fast), G.alloc_work(m, n, k, N, ct), ct)
    torch.cuda.synchronize()
    out[name + "_ref"], out[name + "_new"] = Cr.cpu().numpy(), Cn.cpu().numpy()
    print(name, "bytes differ", int((Cr.view(torch.uint8) != Cn.view(torch.uint8)).sum()), flush=True)
out["c0"] = C0.cpu().numpy()
out["ab"] = np.array([al, be])
np.savez(os.path.join(ROOT, "gpurun_out", os.environ.get("DUMP", "epi_dump2") + ".npz"), **out)
