"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU restatement (oz2_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It is the checker, never the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboz2oracle.so")
_lib = None

_TCODE = {np.float64: "d", np.float32: "s", np.complex128: "z", np.complex64: "c"}


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        p, sz, u, i, c = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_int, ctypes.c_char
        _lib.oz2o_scaling.argtypes = [c, c, i, i, sz, sz, sz, p, sz, p, sz, u, i, i, p, p, p, p]
        _lib.oz2o_scaling_ex.argtypes = [c, c, i, i, sz, sz, sz, p, sz, p, sz, u, i, i, p, p, p, p, p, p, i]
        _lib.oz2o_residues.argtypes = [sz, sz, sz, u, p, p, p]
        _lib.oz2o_crt.argtypes = [c, i, sz, sz, u, p, p, p, p, p, p, sz, i]
        _lib.oz2o_gemm.argtypes = [c, c, c, i, i, sz, sz, sz, p, p, sz, p, sz, p, p, sz, u, i, i, i, p, p, i]
        _lib.oz2o_vnni.restype = i
        _lib.oz2o_vnni.argtypes = []
        _lib.oz2o_set_num_threads.argtypes = [i]
        _lib.oz2o_set_num_threads.restype = None
    return _lib


def tcode(dtype):
    return _TCODE[np.dtype(dtype).type].encode()


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def default_vt(ta, tb):
    """threads_scaling of the reference entry point (gemmul8.cu:206-222, 349-365, 490-506, 636-652)."""
    return 512 if (ta == np.float32 and tb == np.float32) else 128


def scaling(A, B, num_moduli, fastmode=True, opA=0, opB=0, vt=None, colmax_in=None, want_colmax=False, ctype=None):
    """Returns (A8 [N, mr, kr], B8 [N, n, kr], sftA [m], sftB [n]) for column-major A, B.

    Accurate mode only: colmax_in replaces the bound product's column maxima (row-block
    sharding); want_colmax appends this call's column maxima to the result."""
    A = np.asfortranarray(A)
    B = np.asfortranarray(B)
    m = A.shape[1] if opA else A.shape[0]
    k = A.shape[0] if opA else A.shape[1]
    n = B.shape[0] if opB else B.shape[1]
    cp = np.iscomplexobj(A)
    kr, mr = (2 * k, 2 * m) if cp else (k, m)
    vt = vt or default_vt(A.dtype.type, B.dtype.type)
    A8 = np.zeros((num_moduli, mr, kr), np.int8)
    B8 = np.zeros((num_moduli, n, kr), np.int8)
    sA = np.zeros(m, np.int16)
    sB = np.zeros(n, np.int16)
    cin = None if colmax_in is None else np.ascontiguousarray(colmax_in, np.int32)
    cout = np.zeros(n, np.int32) if want_colmax else None
    rc = lib().oz2o_scaling_ex(tcode(A.dtype), tcode(B.dtype), opA, opB, m, n, k, _ptr(A), A.shape[0], _ptr(B),
                               B.shape[0], num_moduli, int(fastmode), vt, _ptr(A8), _ptr(B8), _ptr(sA), _ptr(sB),
                               None if cin is None else _ptr(cin), None if cout is None else _ptr(cout),
                               (1 if cp else 0) if ctype is None else ctype)
    if rc:
        raise ValueError(f"oz2o_scaling rc={rc}")
    return (A8, B8, sA, sB, cout) if want_colmax else (A8, B8, sA, sB)


def residues(A8, B8):
    N, mr, kr = A8.shape
    n = B8.shape[1]
    R = np.zeros((N, n, mr), np.uint8)  # plane j: column-major mr x n
    lib().oz2o_residues(mr, n, kr, N, _ptr(np.ascontiguousarray(A8)), _ptr(np.ascontiguousarray(B8)), _ptr(R))
    return R


def crt(R, sftA, sftB, out_dtype, alpha=1.0, beta=0.0, C=None, quirks=False):
    N, n, mr = R.shape
    cp = np.issubdtype(np.dtype(out_dtype), np.complexfloating)
    m = mr // 2 if cp else mr
    if C is None:
        C = np.zeros((m, n), out_dtype, order="F")
    C = np.asfortranarray(C.astype(out_dtype))
    al = np.array([alpha], out_dtype)
    be = np.array([beta], out_dtype)
    lib().oz2o_crt(tcode(out_dtype), int(cp), m, n, N, _ptr(np.ascontiguousarray(R)), _ptr(sftA), _ptr(sftB),
                   _ptr(al), _ptr(be), _ptr(C), C.shape[0], int(quirks))
    return C


def gemm(A, B, num_moduli, fastmode=True, out_dtype=None, alpha=1.0, beta=0.0, C=None, opA=0, opB=0,
         vt=None, quirks=False, return_sft=False, ctype=None):
    """C = alpha * op(A) @ op(B) + beta * C through the restated reference pipeline."""
    A = np.asfortranarray(A)
    B = np.asfortranarray(B)
    out_dtype = out_dtype or np.result_type(A.dtype, B.dtype)
    m = A.shape[1] if opA else A.shape[0]
    k = A.shape[0] if opA else A.shape[1]
    n = B.shape[0] if opB else B.shape[1]
    vt = vt or default_vt(A.dtype.type, B.dtype.type)
    if C is None:
        C = np.zeros((m, n), out_dtype, order="F")
    C = np.asfortranarray(C.astype(out_dtype))
    al = np.array([alpha], out_dtype)
    be = np.array([beta], out_dtype)
    sA = np.zeros(m, np.int16)
    sB = np.zeros(n, np.int16)
    rc = lib().oz2o_gemm(tcode(A.dtype), tcode(B.dtype), tcode(out_dtype), opA, opB, m, n, k, _ptr(al), _ptr(A),
                         A.shape[0], _ptr(B), B.shape[0], _ptr(be), _ptr(C), C.shape[0], num_moduli, int(fastmode),
                         vt, int(quirks), _ptr(sA), _ptr(sB), 0 if ctype is None else ctype)
    if rc:
        raise ValueError(f"oz2o_gemm rc={rc}")
    return (C, sA, sB) if return_sft else C


def num_threads():
    return lib().oz2o_num_threads()


def set_num_threads(n):
    """OpenMP team size of later oracle calls (the bench's CPU baseline; n <= 0: unchanged)"""
    lib().oz2o_set_num_threads(int(n))


def vnni():
    """whether the int8 products take the AVX-512 VNNI path (exact either way; OZ2O_SCALAR=1 forces scalar)"""
    return bool(lib().oz2o_vnni())
