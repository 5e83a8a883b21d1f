"""Dump the unscaled-by-alpha product v (alpha = 1, beta = 0 call, identical in both libraries), C0 and
the reference's / this library's C for complex alpha / beta, to pin the reference's epilogue formula
on the host (probe).  Writes gpurun_out/epi_dump.npz."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mixed-gemmul8_amd")]
import gemmul8 as G
from test_ref_parity import _ref, CODES

lib = _ref()
out = {}
m, n, k, N = 96, 80, 256, 6
for tc, tdt, npt in (("c", torch.complex64, np.complex64), ("z", torch.complex128, np.complex128)):
    A = G.randmat(m, k, tdt, 0.5, 11)
    B = G.randmat(k, n, tdt, 0.5, 12)
    C0 = G.randmat(m, n, tdt, 0.5, 13)
    W = G.alloc_work(m, n, k, N, 1)
    V = torch.zeros_like(C0)
    G.gemm(0, 0, m, n, k, complex(1), A, m, B, k, complex(0), V, m, N, True, W, 1)
    for name, al, be in (("a", 1.5 - 0.5j, 0), ("ab", 1.5 - 0.5j, 0.25 + 0.75j), ("a1", 1 + 1j, 1), ("r1", 2.5, 1),
                         ("rb", 2.5, 0.5)):
        Cr, Cn = C0.clone(), C0.clone()
        alpha, beta = np.array([al], npt), np.array([be], npt)
        w = torch.zeros(lib.ref_work_size(m, n, k, N, 1) + (1 << 22), dtype=torch.uint8, device="cuda")
        rc = lib.ref_gemm(CODES[tc], CODES[tc], CODES[tc], 0, 0, m, n, k, alpha.ctypes.data, A.data_ptr(), m,
                          B.data_ptr(), k, beta.ctypes.data, Cr.data_ptr(), m, N, 1, 1, w.data_ptr(), None)
        assert rc == 0
        G.gemm(0, 0, m, n, k, complex(al), A, m, B, k, complex(be), Cn, m, N, True, W, 1)
        torch.cuda.synchronize()
        out[f"{tc}_{name}_ref"] = Cr.cpu().numpy()
        out[f"{tc}_{name}_new"] = Cn.cpu().numpy()
        out[f"{tc}_{name}_ab"] = np.array([al, be], np.complex128)
        print(tc, name, "bytes differ", int((Cr.view(torch.uint8) != Cn.view(torch.uint8)).sum()), flush=True)
    out[f"{tc}_v"] = V.cpu().numpy()
    out[f"{tc}_c0"] = C0.cpu().numpy()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "epi_dump.npz"), **out)
