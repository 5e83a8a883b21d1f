#!/usr/bin/env python3
"""Golden vectors for the BLAS epilogue with general and complex alpha / beta, from the REFERENCE's own
HIP build (oracle/_ref/libgemmul8_ref.so, see make_golden.py) on an MI355X: inputs, C0, alpha, beta and
the reference's C for its _a1 / _ab / CAdd kernels (inverse_scaling.hpp:268-948), real and complex,
one- and two-level moduli.  The reference's non-BLAS variants (_1b; _2_a1; beta = 0 reading C) are left
out.

Run on the GPU box:  python tests/golden/make_golden_epilogue.py <out.npz>
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from util import randmat_np  # noqa: E402

LIB = os.path.join(ROOT, "oracle", "_ref", "libgemmul8_ref.so")
NPT = {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}
CODE = {"d": 0, "s": 1, "z": 2, "c": 3}


def cases():
    out = []
    cplx_ab = [(1.5 - 0.5j, 0.25 + 0.75j), (1.0 + 1.0j, 1.0), (0.3 + 1.7j, -1.25 + 0.5j), (2.5, 0.5), (1.0, 1.0),
               (2.5, -0.5j)]
    for t, N in (("z", 6), ("z", 14), ("c", 8)):
        for i, (al, be) in enumerate(cplx_ab):
            if t == "z" and N == 14 and be == 1.0 and al != 1.0:
                continue  # _2_a1 (non-BLAS)
            out.append((f"{t}_N{N}_ab{i}", t, N, al, be))
    for t, N in (("d", 6), ("d", 14), ("s", 8)):
        for i, (al, be) in enumerate([(2.5, 0.5), (1.0, 1.0), (-0.75, 1.0), (3.0, -2.0)]):
            if t == "d" and N == 14 and be == 1.0 and al != 1.0:
                continue
            out.append((f"{t}_N{N}_ab{i}", t, N, al, be))
    return out


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "golden_epilogue.npz")
    lib = ctypes.CDLL(LIB)
    p, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    lib.ref_gemm.argtypes = [i, i, i, i, i, sz, sz, sz, p, p, sz, p, sz, p, p, sz, u, i, i, p, p]
    lib.ref_work_size.restype = sz
    lib.ref_work_size.argtypes = [sz, sz, sz, u, i]
    m, n, k = 36, 28, 52
    data = {}
    for ci, (name, t, N, al, be) in enumerate(cases()):
        rng = np.random.default_rng(7000 + ci)
        A, B, C0 = randmat_np(rng, m, k, dtype=NPT[t]), randmat_np(rng, k, n, dtype=NPT[t]), randmat_np(rng, m, n, dtype=NPT[t])
        ct = 1 if t in "zc" else 0
        work = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + (1 << 22), dtype=torch.uint8, device="cuda")
        dA = torch.from_numpy(np.ascontiguousarray(A.T)).cuda()
        dB = torch.from_numpy(np.ascontiguousarray(B.T)).cuda()
        dC = torch.from_numpy(np.ascontiguousarray(C0.T)).cuda()
        alpha, beta = np.array([al], NPT[t]), np.array([be], NPT[t])
        rc = lib.ref_gemm(CODE[t], CODE[t], CODE[t], 0, 0, m, n, k, alpha.ctypes.data, dA.data_ptr(), m, dB.data_ptr(),
                          k, beta.ctypes.data, dC.data_ptr(), m, N, 1, ct, work.data_ptr(), None)
        torch.cuda.synchronize()
        C = np.asfortranarray(dC.cpu().numpy().T)
        for key, val in (("A", A), ("B", B), ("C0", C0), ("C", C), ("alpha", alpha), ("beta", beta),
                         ("N", np.array([N], np.int64)), ("rc", np.array([rc], np.int64))):
            data[f"{name}/{key}"] = val
        print(f"{name}: rc={rc}", flush=True)
    np.savez_compressed(out, **data)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
