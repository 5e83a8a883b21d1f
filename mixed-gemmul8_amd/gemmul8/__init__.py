"""gemmul8 -- Python host binding of the MI355X-native Ozaki-scheme-II GEMM emulator.

Thin ctypes layer over the C ABI in ``include/gemmul8_c.h`` (libgemmul8_amd.so,
built in-tree by ``make -C mixed-gemmul8_amd``).  Mirrors the reference C++ API
(GEMMul8/include/gemmul8.hpp:7-287): ``workSize`` and ``gemm`` with the same
argument meaning (column-major device operands, leading dimensions, host
alpha/beta, caller-owned workspace), plus ``matmul`` for row-major torch tensors.
PyTorch is used only for device memory and streams.

There is no CPU fallback: importing this module on a machine without the built
library raises, and every call goes to the HIP kernels.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgemmul8_amd.so")

REAL_DEFAULT, COMPLEX_BIG_MATRIX_ENCODE, COMPLEX_CLASSIC_MULT, COMPLEX_KARATSUBA_MULT = 0, 1, 2, 3
OP_N, OP_T, OP_C = 0, 1, 2
R_64F, R_32F, C_64F, C_32F = 0, 1, 2, 3
_DTYPE = {torch.float64: R_64F, torch.float32: R_32F, torch.complex128: C_64F, torch.complex64: C_32F}
_ERR = {-1: "num_moduli outside [2, 20]", -2: "unsupported dtype combination for computeType",
        -3: "unsupported transpose op", -4: "size limit (padded k beyond 2^22 fast / 2^19 accurate, or leading dimension too small)",
        -5: "mode not implemented in this build", -6: "HIP launch failure"}


class Gemmul8Error(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"gemmul8: native library not built ({LIB_PATH}); run `make -C mixed-gemmul8_amd`")
    lib = ctypes.CDLL(LIB_PATH)
    p, sz, u, i, d = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_int, ctypes.POINTER(ctypes.c_double)
    lib.gemmul8_work_size.restype = sz
    lib.gemmul8_work_size.argtypes = [sz, sz, sz, u, i]
    lib.gemmul8_gemm.restype = i
    lib.gemmul8_gemm.argtypes = [p, i, i, sz, sz, sz, i, i, i, p, p, sz, p, sz, p, p, sz, u, i, p, i, d]
    lib.gemmul8_split.argtypes = [p, i, i, sz, sz, sz, i, i, i, p, sz, p, sz, u, i, p, i, u, u, i]
    lib.gemmul8_split_bound.argtypes = [p, i, i, sz, sz, sz, i, i, i, p, sz, p, sz, u, p, i]
    lib.gemmul8_products.argtypes = [p, sz, sz, sz, u, i, p, u, u]
    lib.gemmul8_recombine.argtypes = [p, sz, sz, sz, u, i, i, p, p, p, sz, p]
    lib.gemmul8_shard_stats.argtypes = [p, i, i, sz, sz, sz, i, i, i, p, sz, p, sz, u, i, p, i, sz, sz, sz, sz]
    lib.gemmul8_shard_bound.argtypes = [p, i, i, sz, sz, sz, i, i, i, p, sz, p, sz, u, p, i, sz, sz]
    lib.gemmul8_products_cols.argtypes = [p, sz, sz, sz, u, i, p, u, u, sz, sz]
    lib.gemmul8_recombine_cols.argtypes = [p, sz, sz, sz, u, i, i, p, p, p, sz, p, sz, sz]
    lib.gemmul8_crt_partial.argtypes = [p, sz, sz, sz, u, i, i, p, u, u, p, sz]
    lib.gemmul8_crt_finish.argtypes = [p, sz, sz, sz, u, i, i, p, p, p, sz, p, p, sz]
    lib.gemmul8_work_size_lowmem.restype = sz
    lib.gemmul8_work_size_lowmem.argtypes = [sz, sz, sz, u, i, u]
    lib.gemmul8_gemm_lowmem.restype = i
    lib.gemmul8_gemm_lowmem.argtypes = [p, i, i, sz, sz, sz, i, i, i, p, p, sz, p, sz, p, p, sz, u, i, p, i, u, d]
    lib.gemmul8_timing_enable.argtypes = [i]
    lib.gemmul8_timing_read.argtypes = [d, ctypes.POINTER(ctypes.c_int)]
    lib.gemmul8_layout.argtypes = [sz, sz, sz, u, i, ctypes.POINTER(ctypes.c_size_t)]
    lib.gemmul8_i8_product_raw.argtypes = [p, sz, sz, sz, u, i, p, p]
    lib.gemmul8_randmat.argtypes = [p, i, sz, sz, p, ctypes.c_double, ctypes.c_ulonglong]
    lib.gemmul8_dd_gemm.argtypes = [p, sz, sz, sz, p, p, p, p]
    lib.gemmul8_relerr_dd.argtypes = [p, sz, p, p, p, p]
    lib.gemmul8_time_gemm.restype = i
    lib.gemmul8_time_gemm.argtypes = [p, i, i, sz, sz, sz, i, i, i, p, p, sz, p, sz, p, p, sz, u, i, p, i, i, d, d]
    lib.gemmul8_time_vendor_gemm.restype = i
    lib.gemmul8_time_vendor_gemm.argtypes = [p, i, sz, sz, sz, p, p, p, i, d]
    lib.gemmul8_set_epilogue.argtypes = [i]
    lib.gemmul8_set_epilogue.restype = i
    lib.gemmul8_get_epilogue.argtypes = []
    lib.gemmul8_get_epilogue.restype = i
    lib.gemmul8_last_products_kernel.restype = ctypes.c_char_p
    lib.gemmul8_last_products_kernel.argtypes = []
    lib.gemmul8_mfma_ceiling.restype = ctypes.c_double
    lib.gemmul8_mfma_ceiling.argtypes = [p, i]
    return lib


lib = _load()


def _stream(stream=None):
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _check(rc):
    if rc != 0:
        raise Gemmul8Error(f"gemmul8 error {rc}: {_ERR.get(rc, 'unknown')}")


class _HostScalar:
    """host alpha/beta buffer of the output type (a ctypes object: a numpy array costs ~3 us per call)"""
    __slots__ = ("buf", "ptr")

    def __init__(self, x, dtype):
        if dtype in (torch.complex128, torch.complex64):
            x = complex(x)
            self.buf = ((ctypes.c_double if dtype == torch.complex128 else ctypes.c_float) * 2)(x.real, x.imag)
        elif dtype == torch.float64:
            self.buf = ctypes.c_double(x)
        elif dtype == torch.float32:
            self.buf = ctypes.c_float(x)
        else:
            raise KeyError(dtype)
        self.ptr = ctypes.addressof(self.buf)


def _scalar(x, dtype):
    return _HostScalar(x, dtype)


def workSize(m, n, k, num_moduli, computeType=REAL_DEFAULT, slice_planes=None):
    """Bytes of device workspace for gemm (gemmul8.hpp:18-22); slice_planes: low-memory mode."""
    if slice_planes:
        return int(lib.gemmul8_work_size_lowmem(m, n, k, num_moduli, computeType, slice_planes))
    return int(lib.gemmul8_work_size(m, n, k, num_moduli, computeType))


def layout(m, n, k, num_moduli, computeType=REAL_DEFAULT):
    out = (ctypes.c_size_t * 24)()
    lib.gemmul8_layout(m, n, k, num_moduli, computeType, out)
    keys = ["m_pad", "n_pad", "k_pad", "ksteps", "planeA", "planeB", "planeR", "offA", "offB", "offR", "offSftA",
            "offSftB", "offBound", "offSft0", "total", "kblk", "ldr", "nsub", "subA", "subB", "subR", "vsA", "vsB",
            "bm_pad"]
    return dict(zip(keys, list(out)))


def gemm(opA, opB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, num_moduli, fastmode, work,
         computeType=REAL_DEFAULT, stream=None, phase_times=False, slice_planes=None):
    """C = alpha*op(A)*op(B) + beta*C on column-major device buffers (gemmul8.hpp:29-47).

    A, B, C, work: torch tensors (storage in column-major order, ld in elements).
    Returns the 4 phase times in ns when phase_times=True (synchronising), else None.
    """
    ta, tb, tc = _DTYPE[A.dtype], _DTYPE[B.dtype], _DTYPE[C.dtype]
    al, be = _scalar(alpha, C.dtype), _scalar(beta, C.dtype)
    pt = (ctypes.c_double * 4)() if phase_times else None
    if slice_planes:
        rc = lib.gemmul8_gemm_lowmem(_stream(stream), opA, opB, m, n, k, ta, tb, tc, al.ptr, A.data_ptr(),
                                     lda, B.data_ptr(), ldb, be.ptr, C.data_ptr(), ldc, num_moduli,
                                     int(bool(fastmode)), work.data_ptr(), computeType, slice_planes, pt)
    else:
        rc = lib.gemmul8_gemm(_stream(stream), opA, opB, m, n, k, ta, tb, tc, al.ptr, A.data_ptr(), lda,
                              B.data_ptr(), ldb, be.ptr, C.data_ptr(), ldc, num_moduli, int(bool(fastmode)),
                              work.data_ptr(), computeType, pt)
    _check(rc)
    return list(pt) if phase_times else None


def time_gemm(opA, opB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc, num_moduli, fastmode, work, iters,
              computeType=REAL_DEFAULT, stream=None):
    """The reference drivers' timing loop in native code (test_double.cu:422-431): `iters` gemm calls, each
    between two device syncs and the host clock.  Returns (seconds per call, the 4 mean phase times in ns)."""
    ta, tb, tc = _DTYPE[A.dtype], _DTYPE[B.dtype], _DTYPE[C.dtype]
    al, be = _scalar(alpha, C.dtype), _scalar(beta, C.dtype)
    sec, pt = ctypes.c_double(), (ctypes.c_double * 4)()
    _check(lib.gemmul8_time_gemm(_stream(stream), opA, opB, m, n, k, ta, tb, tc, al.ptr, A.data_ptr(), lda,
                                 B.data_ptr(), ldb, be.ptr, C.data_ptr(), ldc, num_moduli, int(bool(fastmode)),
                                 work.data_ptr(), computeType, iters, ctypes.byref(sec), pt))
    return sec.value, list(pt)


def time_vendor_gemm(m, n, k, A, B, C, iters, stream=None):
    """The same loop around hipblasGemmEx (op N / N, alpha 1, beta 0, lda = m, ldb = k, ldc = m) on column-major
    A (m x k), B (k x n), C (m x n) of one dtype: the drivers' DGEMM / SGEMM / CGEMM rows.  Seconds per call."""
    if not (A.dtype == B.dtype == C.dtype):
        raise TypeError("time_vendor_gemm: A, B and C must share one dtype")
    sec = ctypes.c_double()
    _check(lib.gemmul8_time_vendor_gemm(_stream(stream), _DTYPE[C.dtype], m, n, k, A.data_ptr(), B.data_ptr(),
                                        C.data_ptr(), iters, ctypes.byref(sec)))
    return sec.value


# ---- phase entry points (gemm == split + products + recombine; used by gemmul8.dist) ----
SPLIT_BOUND_READY = 1
SPLIT_SHIFTS_READY = 2


def split(opA, opB, m, n, k, A, lda, B, ldb, num_moduli, fastmode, work, out_dtype, mod_begin=0, mod_end=None,
          computeType=REAL_DEFAULT, stream=None, bound_ready=False, shifts_ready=False):
    """Shifts of op(A)/op(B) and the int8 slices of moduli [mod_begin, mod_end) into `work`
    (shifts_ready: the shifts are already in `work`, only the slices are encoded)."""
    mod_end = num_moduli if mod_end is None else mod_end
    flags = (SPLIT_BOUND_READY if bound_ready else 0) | (SPLIT_SHIFTS_READY if shifts_ready else 0)
    _check(lib.gemmul8_split(_stream(stream), opA, opB, m, n, k, _DTYPE[A.dtype], _DTYPE[B.dtype], _DTYPE[out_dtype],
                             A.data_ptr(), lda, B.data_ptr(), ldb, num_moduli, int(bool(fastmode)), work.data_ptr(),
                             computeType, mod_begin, mod_end, flags))


def shard_stats(opA, opB, m, n, k, A, lda, B, ldb, num_moduli, fastmode, work, out_dtype, rows, cols,
                computeType=REAL_DEFAULT, stream=None):
    """Shifts (fast) or sft0 (accurate) of the rows [rows) of op(A) and the columns [cols) of op(B) into `work`."""
    _check(lib.gemmul8_shard_stats(_stream(stream), opA, opB, m, n, k, _DTYPE[A.dtype], _DTYPE[B.dtype],
                                   _DTYPE[out_dtype], A.data_ptr(), lda, B.data_ptr(), ldb, num_moduli,
                                   int(bool(fastmode)), work.data_ptr(), computeType, rows[0], rows[1], cols[0],
                                   cols[1]))


def shard_bound(opA, opB, m, n, k, A, lda, B, ldb, num_moduli, work, out_dtype, cols, computeType=REAL_DEFAULT,
                stream=None):
    """Accurate mode with sft0 assembled: the bound product over the columns [cols) of op(B)."""
    _check(lib.gemmul8_shard_bound(_stream(stream), opA, opB, m, n, k, _DTYPE[A.dtype], _DTYPE[B.dtype],
                                   _DTYPE[out_dtype], A.data_ptr(), lda, B.data_ptr(), ldb, num_moduli,
                                   work.data_ptr(), computeType, cols[0], cols[1]))


def split_bound(opA, opB, m, n, k, A, lda, B, ldb, num_moduli, work, out_dtype, computeType=REAL_DEFAULT,
                stream=None):
    """Accurate mode: bound product maxima into `work`; returns (rowmax [m], colmax [n]) int32 views."""
    _check(lib.gemmul8_split_bound(_stream(stream), opA, opB, m, n, k, _DTYPE[A.dtype], _DTYPE[B.dtype],
                                   _DTYPE[out_dtype], A.data_ptr(), lda, B.data_ptr(), ldb, num_moduli,
                                   work.data_ptr(), computeType))
    L = layout(m, n, k, num_moduli, computeType)
    o = L["offBound"]
    rowmax = work[o:o + 4 * m].view(torch.int32)
    colmax = work[o + 4 * L["bm_pad"]:o + 4 * L["bm_pad"] + 4 * n].view(torch.int32)
    return rowmax, colmax


def products(m, n, k, num_moduli, work, mod_begin=0, mod_end=None, computeType=REAL_DEFAULT, stream=None, cols=None):
    """Residue planes of moduli [mod_begin, mod_end) (one MFMA launch) into `work`; cols=(c0, c1): those
    residue columns only (c0 a multiple of 256, c1 one too or n)."""
    mod_end = num_moduli if mod_end is None else mod_end
    if cols is None:
        _check(lib.gemmul8_products(_stream(stream), m, n, k, num_moduli, computeType, work.data_ptr(), mod_begin,
                                    mod_end))
    else:
        _check(lib.gemmul8_products_cols(_stream(stream), m, n, k, num_moduli, computeType, work.data_ptr(),
                                         mod_begin, mod_end, cols[0], cols[1]))


def recombine(m, n, k, num_moduli, alpha, beta, C, ldc, work, computeType=REAL_DEFAULT, stream=None, cols=None):
    """CRT of all residue planes in `work` + scaling + alpha/beta epilogue into C; cols=(c0, c1): those
    output columns only, C then holding column c0 first."""
    al, be = _scalar(alpha, C.dtype), _scalar(beta, C.dtype)
    if cols is None:
        _check(lib.gemmul8_recombine(_stream(stream), m, n, k, num_moduli, _DTYPE[C.dtype], computeType, al.ptr,
                                     be.ptr, C.data_ptr(), ldc, work.data_ptr()))
    else:
        _check(lib.gemmul8_recombine_cols(_stream(stream), m, n, k, num_moduli, _DTYPE[C.dtype], computeType, al.ptr,
                                          be.ptr, C.data_ptr(), ldc, work.data_ptr(), cols[0], cols[1]))


def crt_partial(m, n, k, num_moduli, out_dtype, work, mod_begin, mod_end, sums, stream=None):
    """Partial CRT sums of moduli [mod_begin, mod_end) into `sums` (float64 tensor (2, n, m): C1 then C2,
    column-major planes; real outputs).  The element-wise sums of the partials of a moduli partition
    finish with crt_finish (include/gemmul8_c.h: C1 exact, C2 rounded in the summation order)."""
    _check_sums(sums, m, n)
    _check(lib.gemmul8_crt_partial(_stream(stream), m, n, k, num_moduli, _DTYPE[out_dtype], REAL_DEFAULT,
                                   work.data_ptr(), mod_begin, mod_end, sums.data_ptr(), m))


def _check_sums(sums, m, n):
    """the partial-sum planes the native kernels index as double [2][n][m] (lds = m)"""
    if sums.dtype != torch.float64:
        raise TypeError(f"partial CRT sums must be float64, not {sums.dtype}")
    if not sums.is_contiguous():
        raise ValueError("partial CRT sums must be contiguous (column-major [2][n][m] planes)")
    if sums.numel() < 2 * n * m:
        raise ValueError(f"partial CRT sums hold {sums.numel()} doubles, need 2 * n * m = {2 * n * m}")


def _check_colmajor(name, X, rows, cols, ld):
    """X addresses a column-major rows x cols matrix with leading dimension ld: unit stride within a column,
    ld between columns (a (cols, rows) view of a (cols, ld) tensor, e.g. a sub-matrix), and the storage behind
    the view reaches the last element"""
    if ld < rows:
        raise ValueError(f"{name}: leading dimension {ld} < {rows} rows")
    if rows == 0 or cols == 0:
        return
    col_stride = X.stride(0) if X.dim() == 2 else ld
    if X.dim() not in (1, 2) or X.stride(-1) != 1 or (cols > 1 and X.dim() == 2 and X.shape[0] > 1 and col_stride != ld):
        raise ValueError(f"{name}: shape {tuple(X.shape)} strides {X.stride()} is not a column-major layout with "
                         f"unit row stride and ld = {ld}")
    extent = X.storage_offset() + ld * (cols - 1) + rows
    avail = X.untyped_storage().nbytes() // X.element_size()
    if extent > avail:
        raise ValueError(f"{name}: a column-major {rows} x {cols} matrix with ld = {ld} needs {extent} elements of "
                         f"storage from the view's base, the tensor's storage holds {avail}")


def crt_finish(m, n, k, num_moduli, alpha, beta, C, ldc, work, sums, stream=None, out_dtype=None):
    """C = alpha * CRT(summed partials) scaled by the workspace's shifts + beta * C (real outputs).
    C: a column-major m x n matrix with leading dimension ldc (any view with unit row stride and column stride
    ldc, as gemm() accepts).  out_dtype: the output type crt_partial was called with, checked against C's."""
    _check_sums(sums, m, n)
    if C.dtype not in (torch.float64, torch.float32):
        raise TypeError(f"crt_finish: C must be float64 or float32, not {C.dtype}")
    if out_dtype is not None and C.dtype != out_dtype:
        raise TypeError(f"crt_finish: C is {C.dtype}, the partial sums were formed for {out_dtype}")
    _check_colmajor("crt_finish: C", C, m, n, ldc)
    al, be = _scalar(alpha, C.dtype), _scalar(beta, C.dtype)
    _check(lib.gemmul8_crt_finish(_stream(stream), m, n, k, num_moduli, _DTYPE[C.dtype], REAL_DEFAULT, al.ptr, be.ptr,
                                  C.data_ptr(), ldc, work.data_ptr(), sums.data_ptr(), m))


def residue_planes(work, m, n, k, num_moduli, mod_begin=0, mod_end=None, computeType=REAL_DEFAULT):
    """uint8 view [mod_end - mod_begin, planeR] of the residue planes inside `work` (no copy)."""
    mod_end = num_moduli if mod_end is None else mod_end
    L = layout(m, n, k, num_moduli, computeType)
    start = L["offR"] + mod_begin * L["planeR"]
    return work[start:start + (mod_end - mod_begin) * L["planeR"]].view(mod_end - mod_begin, L["planeR"])


def alloc_work(m, n, k, num_moduli, computeType=REAL_DEFAULT, device="cuda", slice_planes=None):
    return torch.empty(workSize(m, n, k, num_moduli, computeType, slice_planes), dtype=torch.uint8, device=device)


def matmul(A, B, num_moduli=14, fastmode=True, out_dtype=None, work=None):
    """Row-major torch convenience: returns A @ B emulated with num_moduli int8 products.

    A row-major (m x k) tensor is a column-major k x m matrix, so the call uses
    op T on both operands and needs no copies."""
    assert A.is_cuda and B.is_cuda and A.dim() == 2 and B.dim() == 2 and A.shape[1] == B.shape[0]
    A = A.contiguous()
    B = B.contiguous()
    m, k = A.shape
    n = B.shape[1]
    out_dtype = out_dtype or torch.promote_types(A.dtype, B.dtype)
    cplx = A.is_complex()
    ct = COMPLEX_BIG_MATRIX_ENCODE if cplx else REAL_DEFAULT
    Ct = torch.empty((n, m), dtype=out_dtype, device=A.device)  # column-major m x n
    if work is None:
        work = alloc_work(m, n, k, num_moduli, ct, A.device)
    if cplx:
        # complex: materialise column-major operands so the call is op N x op N, the form a BLAS
        # caller (and the interposer) passes for a row-major product; its bits then match it
        Acm = A.t().contiguous()
        Bcm = B.t().contiguous()
        gemm(OP_N, OP_N, m, n, k, 1.0, Acm, m, Bcm, k, 0.0, Ct, m, num_moduli, fastmode, work, ct)
    else:
        gemm(OP_T, OP_T, m, n, k, 1.0, A, k, B, n, 0.0, Ct, m, num_moduli, fastmode, work, ct)
    return Ct.t()


# ---- instrumentation ----
def timing_enable(on=True):
    lib.gemmul8_timing_enable(1 if on else 0)


def timing_read():
    ms = (ctypes.c_double * 4)()
    calls = ctypes.c_int(0)
    lib.gemmul8_timing_read(ms, ctypes.byref(calls))
    return list(ms), calls.value


# ---- harness (reference test-driver semantics) ----
def randmat(m, n, dtype=torch.float64, phi=0.5, seed=123456, device="cuda", stream=None):
    """Column-major m x n matrix (returned as an (n, m) row-major tensor) from make_matrix.hpp:8-71."""
    X = torch.empty((n, m), dtype=dtype, device=device)
    _check(lib.gemmul8_randmat(_stream(stream), _DTYPE[dtype], m, n, X.data_ptr(), phi, seed))
    return X


def dd_gemm(Acm, Bcm, m, n, k, stream=None):
    """double-double reference of column-major A (m x k) * B (k x n); returns (C1, C2) column-major."""
    C1 = torch.empty((n, m), dtype=torch.float64, device=Acm.device)
    C2 = torch.empty_like(C1)
    _check(lib.gemmul8_dd_gemm(_stream(stream), m, n, k, Acm.data_ptr(), Bcm.data_ptr(), C1.data_ptr(),
                               C2.data_ptr()))
    return C1, C2


def relerr_dd(C, C1, C2, stream=None):
    """elementwise |C - C1 - C2| / |C1 + C2| in double-double, returns (max, median) like eval.hpp:317-338."""
    err = torch.empty(C1.numel(), dtype=torch.float64, device=C1.device)
    _check(lib.gemmul8_relerr_dd(_stream(stream), C1.numel(), C.data_ptr(), C1.data_ptr(), C2.data_ptr(),
                                 err.data_ptr()))
    s, _ = torch.sort(err)
    cnt = s.numel()
    med = s[cnt // 2] if cnt & 1 else (s[cnt // 2] + s[cnt // 2 - 1]) * 0.5
    return float(s[-1]), float(med)


EPILOGUE_BLAS, EPILOGUE_REFERENCE = 0, 1


def set_epilogue(mode):
    """Epilogue semantics for later calls: "blas" (default) or "reference" (the reference's kernels bit for bit,
    their non-BLAS alpha / beta variants included; include/gemmul8_c.h).  Returns the previous mode's name."""
    names = {"blas": EPILOGUE_BLAS, "reference": EPILOGUE_REFERENCE}
    prev = get_epilogue()
    _check(lib.gemmul8_set_epilogue(names[mode] if isinstance(mode, str) else int(mode)))
    return prev


def get_epilogue():
    return "reference" if lib.gemmul8_get_epilogue() == EPILOGUE_REFERENCE else "blas"


def last_products_kernel():
    """name of the residue-product kernel the last products launch of this process took"""
    return lib.gemmul8_last_products_kernel().decode()


def mfma_ceiling(iters=4000, stream=None):
    """TOPS of the int8 MFMA alone (the better of 32x32x32 and 16x16x64) on uniformly random operand
    bytes: the data-bound ceiling of the int8 products at the clock the GPU holds under that load."""
    return float(lib.gemmul8_mfma_ceiling(_stream(stream), iters))
