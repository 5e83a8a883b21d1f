#!/usr/bin/env python3
"""Golden vectors for the complex compute types, from the REFERENCE's own HIP build
(oracle/_ref/libgemmul8_ref.so, see make_golden.py) on an MI355X.

Covers COMPLEX_BIG_MATRIX_ENCODE (1), COMPLEX_CLASSIC_MULT (2) and COMPLEX_KARATSUBA_MULT (3),
fast and accurate mode, op N / T / C on either side, complex-double and complex-float
operands.  Stores inputs, C and the reference's sftA / sftB (workspace layouts:
GEMMul8/src/gemmul8.cu:612-664 big matrix, :760-823 Karatsuba, :925-990 classic).

Run on the GPU box:  python tests/golden/make_golden_complex.py <out.npz>
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
NPT = {"z": np.complex128, "c": np.complex64}
TC = {"z": 2, "c": 3}


def pad16(x):
    return (x + 15) // 16 * 16


def sft_offsets(m, n, k, N, ctype):
    if ctype == 1:  # big matrix (HIP branch)
        k2 = pad16(2 * k)
        lda8i = k2 + 64 if k2 % 1024 == 0 else k2
        m_pad = 2 * m
        sizeC = pad16(m_pad * n)
        sizeC32i = pad16(2 * (m + 1) * n) if m % 512 == 0 else pad16(m_pad * n)
        sizeA, sizeB = lda8i * m_pad, lda8i * n
        off = N * (sizeA + sizeB) + N * sizeC + 4 * sizeC32i
    else:  # classic / Karatsuba (HIP branch)
        k16 = pad16(k)
        lda8i = k16 + 64 if k16 % 1024 == 0 else k16
        sizeA, sizeB = lda8i * m, lda8i * n
        sizeC = pad16(m * n)
        sizeC32i = pad16((m + 1) * n) if m % 1024 == 0 else sizeC
        off = 2 * N * (sizeA + sizeB) + 2 * N * sizeC + 2 * 4 * sizeC32i
    return off, off + 2 * pad16(m)


def cases():
    out = []
    ops = [(0, 0), (1, 0), (2, 0), (0, 1), (0, 2), (1, 2), (2, 1)]
    for ctype in (1, 2, 3):
        for fast in (1, 0):
            for opA, opB in ops:
                out.append((f"zzz_ct{ctype}_{'fast' if fast else 'accu'}_op{opA}{opB}", "z", "z", "z", opA, opB,
                            37, 29, 45, 12, fast, ctype))
        out.append((f"ccc_ct{ctype}_fast_op00", "c", "c", "c", 0, 0, 40, 24, 33, 8, 1, ctype))
        out.append((f"ccc_ct{ctype}_accu_op00", "c", "c", "c", 0, 0, 40, 24, 33, 7, 0, ctype))
        out.append((f"zcz_ct{ctype}_fast_op10", "z", "c", "z", 1, 0, 30, 26, 40, 10, 1, ctype))
        out.append((f"zzz_ct{ctype}_fast_N20", "z", "z", "z", 0, 0, 24, 20, 70, 20, 1, ctype))
    # accurate mode, op C pinned where the reference is deterministic and correct: square shapes
    # for op(A) = C (big matrix), complex-float output for classic / Karatsuba (their C is written)
    out.append(("zzz_ct1_accu_op20_sq", "z", "z", "z", 2, 0, 33, 33, 44, 12, 0, 1))
    out.append(("zzz_ct1_accu_op22_sq", "z", "z", "z", 2, 2, 33, 33, 45, 12, 0, 1))
    out.append(("ccc_ct1_accu_op22_sq", "c", "c", "c", 2, 2, 40, 40, 36, 7, 0, 1))
    out.append(("zzz_ct1_accu_op02_k0", "z", "z", "z", 0, 2, 37, 29, 48, 12, 0, 1))
    for ctype in (2, 3):
        for opA, opB in ((1, 0), (0, 1), (0, 2), (1, 2)):
            out.append((f"ccc_ct{ctype}_accu_op{opA}{opB}", "c", "c", "c", opA, opB, 40, 24, 36, 7, 0, ctype))
    return out


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "golden_complex.npz")
    lib = ctypes.CDLL(LIB)
    p, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    lib.ref_gemm.argtypes = [i, i, i, i, i, sz, sz, sz, p, p, sz, p, sz, p, p, sz, u, i, i, p, p]
    lib.ref_work_size.restype = sz
    lib.ref_work_size.argtypes = [sz, sz, sz, u, i]
    data = {}
    for ci, (name, ta, tb, tc, opA, opB, m, n, k, N, fast, ctype) in enumerate(cases()):
        rng = np.random.default_rng(5000 + ci)
        A = randmat_np(rng, k, m, dtype=NPT[ta]) if opA else randmat_np(rng, m, k, dtype=NPT[ta])
        B = randmat_np(rng, n, k, dtype=NPT[tb]) if opB else randmat_np(rng, k, n, dtype=NPT[tb])
        ws = lib.ref_work_size(m, n, k, N, ctype)
        work = torch.zeros(ws + 16 * A.size + 16 * B.size + (1 << 20), dtype=torch.uint8, device="cuda")
        dA = torch.from_numpy(np.ascontiguousarray(A.T)).cuda()
        dB = torch.from_numpy(np.ascontiguousarray(B.T)).cuda()
        dC = torch.zeros((n, m), dtype=torch.from_numpy(np.zeros(1, NPT[tc])).dtype, device="cuda")
        one = np.array([1], NPT[tc])
        zero = np.array([0], NPT[tc])
        rc = lib.ref_gemm(TC[ta], TC[tb], TC[tc], opA, opB, m, n, k, one.ctypes.data, dA.data_ptr(), A.shape[0],
                          dB.data_ptr(), B.shape[0], zero.ctypes.data, dC.data_ptr(), m, N, fast, ctype,
                          work.data_ptr(), None)
        torch.cuda.synchronize()
        C = np.asfortranarray(dC.cpu().numpy().T)
        wsb = work.cpu().numpy()
        oA, oB = sft_offsets(m, n, k, N, ctype)
        opa = {0: lambda X: X, 1: lambda X: X.T, 2: lambda X: X.conj().T}
        exact = opa[opA](A.astype(np.complex128)) @ opa[opB](B.astype(np.complex128))
        err = float(np.max(np.abs(C - exact) / np.maximum(np.abs(exact), 1e-300)))
        data[f"{name}/A"] = A
        data[f"{name}/B"] = B
        data[f"{name}/C"] = C
        data[f"{name}/sftA"] = wsb[oA:oA + 2 * m].view(np.int16).copy()
        data[f"{name}/sftB"] = wsb[oB:oB + 2 * n].view(np.int16).copy()
        data[f"{name}/meta"] = np.array([opA, opB, m, n, k, N, fast, ctype], np.int64)
        data[f"{name}/types"] = np.array([ta + tb + tc])
        data[f"{name}/rc"] = np.array([rc], np.int64)
        print(f"{name}: rc={rc} max relerr {err:.3e}", flush=True)
    np.savez_compressed(out, **data)
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
