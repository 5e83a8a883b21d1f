"""Element-level view of live fuzz failures: positions, values of both implementations and of C0 (probe).
python fuzz_ref_elems.py failures.json [count] [per-case elements]"""
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
cnt = int(sys.argv[2]) if len(sys.argv) > 2 else 6
per = int(sys.argv[3]) if len(sys.argv) > 3 else 4
seen = set()
for f in fails:
    key = (f["types"][2], f["alpha"], f["beta"], f["fast"])
    if key in seen:
        continue
    seen.add(key)
    if len(seen) > cnt:
        break
    ta, tb, tc = f["types"]
    m, n, k, N, fast, ct = f["m"], f["n"], f["k"], f["N"], f["fast"], f["ct"]
    opA, opB = f["op"]
    seed, phi = f["seed"], f["phi"]
    # regenerate exactly as fuzz_ref did: its rng draws for the special injection are not reproducible
    # here, so rerun with the special inputs rebuilt from a fresh rng keyed on the seed
    rng = np.random.default_rng(seed)
    A = G.randmat(k, m, F.TDT[ta], phi, seed) if opA else G.randmat(m, k, F.TDT[ta], phi, seed)
    B = G.randmat(n, k, F.TDT[tb], phi, seed + 1) if opB else G.randmat(k, n, F.TDT[tb], phi, seed + 1)
    dbl = lambda t: t in "dz"
    for X, t, axis, nv in ((A, ta, 0 if opA else 1, m), (B, tb, 1 if opB else 0, n)):
        if nv >= 6 and X.shape[0] >= 2 and X.shape[1] >= 2:
            _extreme(X, axis, *((1e200, 1e-200, 1e-310) if dbl(t) else (1e25, 1e-25, 1e-40)))
    C0 = G.randmat(m, n, F.TDT[tc], 0.5, seed + 2)
    lda, ldb = (k if opA else m), (n if opB else k)
    C_ref, C_new = C0.clone(), C0.clone()
    alpha, beta = np.array([f["alpha"]], F.NPT[tc]), np.array([f["beta"]], F.NPT[tc])
    w = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + 16 * max(A.numel(), B.numel()) + (1 << 20), dtype=torch.uint8, device="cuda")
    lib.ref_gemm(CODES[ta], CODES[tb], CODES[tc], opA, opB, m, n, k, alpha.ctypes.data, A.data_ptr(), lda, B.data_ptr(), ldb,
                 beta.ctypes.data, C_ref.data_ptr(), m, N, fast, ct, w.data_ptr(), None)
    cplx = ta in "cz"
    G.gemm(opA, opB, m, n, k, complex(f["alpha"]) if cplx else f["alpha"], A, lda, B, ldb,
           complex(f["beta"]) if cplx else f["beta"], C_new, m, N, bool(fast), G.alloc_work(m, n, k, N, ct), ct)
    torch.cuda.synchronize()
    R = C_ref.view(torch.uint8).view(n, m, -1); W = C_new.view(torch.uint8).view(n, m, -1)
    d = (R != W).any(-1)
    idx = torch.nonzero(d)
    print(f, "elements differing:", int(d.sum()), flush=True)
    for j, i in idx[:per].tolist():
        print(f"   C[{i},{j}] ref {C_ref[j, i].item()!r} new {C_new[j, i].item()!r} C0 {C0[j, i].item()!r}")
