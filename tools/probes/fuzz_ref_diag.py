"""Accuracy of the reference's and this library's C on the fuzz_ref failures (probe)."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mixed-gemmul8_amd"), os.path.dirname(__file__)]
import gemmul8 as G
from test_ref_parity import _ref, CODES
from fuzz_ref import TDT, NPT

lib = _ref()
cases = json.load(open(sys.argv[1]))["failures"]
for f in cases[:int(sys.argv[2]) if len(sys.argv) > 2 else 8]:
    ta, tb, tc = f["types"]
    m, n, k, N, fast, ct = f["m"], f["n"], f["k"], f["N"], f["fast"], f["ct"]
    opA, opB = f["op"]
    seed, phi = f["seed"], f["phi"]
    A = G.randmat(k, m, TDT[ta], phi, seed) if opA else G.randmat(m, k, TDT[ta], phi, seed)
    B = G.randmat(n, k, TDT[tb], phi, seed + 1) if opB else G.randmat(k, n, TDT[tb], phi, seed + 1)
    lda, ldb = (k if opA else m), (n if opB else k)
    for variant in ("as-is", "opN-copies"):
        if variant == "opN-copies":  # the same product with op N operands (materialised op(A), op(B))
            opAm = A.t() if opA == 0 else (A.conj() if opA == 2 else A)  # row-major m x k of op(A)
            opBm = (B.conj() if opB == 2 else B) if opB else B.t()  # row-major k x n of op(B)
            A2 = opAm.t().contiguous()  # (k, m) tensor = column-major m x k
            B2 = opBm.t().contiguous()  # (n, k) tensor = column-major k x n
            args = (0, 0, A2, m, B2, k)
        else:
            args = (opA, opB, A, lda, B, ldb)
        oa, ob, AA, la, BB, lb = args
        C_ref = torch.zeros((n, m), dtype=TDT[tc], device="cuda"); C_new = torch.zeros_like(C_ref)
        one, zero = np.array([1], NPT[tc]), np.array([0], NPT[tc])
        w = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + 16 * max(A.numel(), B.numel()) + (1 << 20), dtype=torch.uint8, device="cuda")
        lib.ref_gemm(CODES[ta], CODES[tb], CODES[tc], oa, ob, m, n, k, one.ctypes.data, AA.data_ptr(), la, BB.data_ptr(), lb,
                     zero.ctypes.data, C_ref.data_ptr(), m, N, fast, ct, w.data_ptr(), None)
        G.gemm(oa, ob, m, n, k, 1.0, AA, la, BB, lb, 0.0, C_new, m, N, bool(fast), G.alloc_work(m, n, k, N, ct), ct)
        # exact: row-major op(A) (m x k) @ op(B) (k x n)
        opA_rm = AA.t() if oa == 0 else (AA.conj() if oa == 2 else AA)
        opB_rm = BB.t() if ob == 0 else (BB.conj() if ob == 2 else BB)
        X = (opA_rm.to(torch.complex128) @ opB_rm.to(torch.complex128)).t()  # (n, m) col-major C
        def err(C):
            e = (C.to(torch.complex128) - X).abs() / X.abs()
            return float(e.max()), float(e.median())
        nd = int((C_ref.view(torch.uint8) != C_new.view(torch.uint8)).sum())
        print(f["types"], m, n, k, "N", N, "op", f["op"], "phi", phi, variant, "diff bytes", nd, "ref err", err(C_ref), "new err", err(C_new), flush=True)
