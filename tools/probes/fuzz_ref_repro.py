"""Re-run one live-fuzz case (fuzz_ref.py's desc, special inputs included) and print where the two
libraries' C differ, with shifts' worth of context (probe).  python fuzz_ref_repro.py failures.json [i ...]"""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mixed-gemmul8_amd"), os.path.dirname(__file__)]
import gemmul8 as G
from test_ref_parity import _ref, _extreme, CODES
import fuzz_ref as F

lib = _ref()
fails = json.load(open(sys.argv[1]))["failures"]
which = [int(x) for x in sys.argv[2:]] or range(len(fails))
for t in which:
    f = fails[t]
    ta, tb, tc = f["types"]
    m, n, k, N, fast, ct = f["m"], f["n"], f["k"], f["N"], f["fast"], f["ct"]
    opA, opB = f["op"]
    seed, phi = f["seed"], f["phi"]
    al, be = complex(f["alpha"]), complex(f["beta"])
    cplx = ta in "cz"
    lda, ldb, ldc = f.get("ld") or [k if opA else m, n if opB else k, m]
    A = G.randmat(lda, m if opA else k, F.TDT[ta], phi, seed)
    B = G.randmat(ldb, k if opB else n, F.TDT[tb], phi, seed + 1)
    if f["special"]:
        dbl = lambda t: t in "dz"
        for X, tt, axis, nv in ((A, ta, 0 if opA else 1, m), (B, tb, 1 if opB else 0, n)):
            if nv >= 6 and X.shape[0] >= 2 and X.shape[1] >= 2:
                _extreme(X, axis, *((1e200, 1e-200, 1e-310) if dbl(tt) else (1e25, 1e-25, 1e-40)))
        for w, i, j, val in f.get("inj", []):
            (A if w == "A" else B)[i, j] = float(val)
    C0 = G.randmat(ldc, n, F.TDT[tc], 0.5, seed + 2)
    Cr, Cn = C0.clone(), C0.clone()
    alpha, beta = np.array([al if cplx else al.real], F.NPT[tc]), np.array([be if cplx else be.real], F.NPT[tc])
    w = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + 16 * max(A.numel(), B.numel()) + (1 << 22), dtype=torch.uint8, device="cuda")
    lib.ref_gemm(CODES[ta], CODES[tb], CODES[tc], opA, opB, m, n, k, alpha.ctypes.data, A.data_ptr(), lda, B.data_ptr(), ldb,
                 beta.ctypes.data, Cr.data_ptr(), ldc, N, fast, ct, w.data_ptr(), None)
    G.gemm(opA, opB, m, n, k, al if cplx else al.real, A, lda, B, ldb, be if cplx else be.real, Cn, ldc, N, bool(fast),
           G.alloc_work(m, n, k, N, ct), ct)
    torch.cuda.synchronize()
    # accuracy of both against the FP64 product of the same operands (row-major op(A) @ op(B))
    Am = A[:, :m] if opA else A[:, :m].t()  # (m, k) once opA's conj is applied below
    Am = (A[:, :k].t() if False else None)
    opA_rm = (A[:m, :k] if opA else A[:k, :m].t())
    opA_rm = opA_rm.conj() if opA == 2 else opA_rm
    opB_rm = (B[:n, :k].t() if opB else B[:, :ldb][:, :k].t()) if False else (B[:k, :n] if opB else B[:n, :k].t())
    opB_rm = opB_rm.conj() if opB == 2 else opB_rm
    X = (opA_rm.to(torch.complex128) @ opB_rm.to(torch.complex128)) * al + be * C0[:n, :m].t().to(torch.complex128)
    def err(C):
        e = (C[:n, :m].t().to(torch.complex128) - X).abs() / X.abs()
        return float(e.max()), float(e.median())
    print("   relerr ref", err(Cr), "new", err(Cn))
    Cr, Cn = Cr[:n, :m].contiguous(), Cn[:n, :m].contiguous()
    R = Cr.view(torch.uint8).view(n, m, -1); W = Cn.view(torch.uint8).view(n, m, -1)
    d = (R != W).any(-1)
    rows = torch.nonzero(d.any(0)).flatten().tolist(); cols = torch.nonzero(d.any(1)).flatten().tolist()
    print(t, {k2: f[k2] for k2 in ("types", "m", "n", "k", "N", "fast", "ct", "op", "alpha", "beta", "inj")}, flush=True)
    print("   differing", int(d.sum()), "rows", rows[:10], len(rows), "cols", cols[:10], len(cols))
    for j, i in torch.nonzero(d)[:4].tolist():
        print(f"   C[{i},{j}] ref {Cr[j, i].item()!r} new {Cn[j, i].item()!r} C0 {C0[j, i].item()!r}")
