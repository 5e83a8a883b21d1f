"""The drop-in boundary: libgemmul8_amd.so loads and exports every C entry point declared in
include/gemmul8_c.h, and every C++ symbol of the reference library (identical mangled names, so
objects compiled against the reference's gemmul8.hpp link unchanged).  No GPU needed."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mixed-gemmul8_amd", "gemmul8", "libgemmul8_amd.so")


def _declared_c_functions():
    with open(os.path.join(ROOT, "include", "gemmul8_c.h")) as f:
        txt = f.read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gemmul8_[a-z0-9_]+)\s*\(", txt)))


def _exported():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_loads():
    assert os.path.exists(LIB), "build first: make -C mixed-gemmul8_amd"
    ctypes.CDLL(LIB)


def test_c_abi_exports_every_declared_function():
    decl = _declared_c_functions()
    assert len(decl) >= 9
    exp = _exported()
    missing = [f for f in decl if f not in exp]
    assert not missing, missing


def test_cpp_symbols_match_reference():
    with open(os.path.join(ROOT, "tests", "golden", "ref_symbols.txt")) as f:
        ref = f.read().split()
    exp = _exported()
    missing = [s for s in ref if s not in exp]
    assert not missing, missing
    assert any("gemmIdddE" in s for s in ref)


def test_work_size_and_errors_host_only():
    lib = ctypes.CDLL(LIB)
    lib.gemmul8_work_size.restype = ctypes.c_size_t
    lib.gemmul8_work_size.argtypes = [ctypes.c_size_t] * 3 + [ctypes.c_uint, ctypes.c_int]
    ws = lib.gemmul8_work_size(8192, 8192, 8192, 14, 0)
    # 14 planes of A and B slices + 14 residue planes + shifts (layout in csrc/oz2_common.hpp)
    assert ws >= 14 * (2 * 8192 * 8192 + 8192 * 8192)
    assert lib.gemmul8_work_size(8192, 8192, 8192, 14, 7) == 0  # unknown compute type (gemmul8.cu:142-145)
    lib.gemmul8_gemm.restype = ctypes.c_int
    # invalid arguments are rejected before anything touches the device
    p = ctypes.c_void_p
    lib.gemmul8_gemm.argtypes = [p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, p, p, ctypes.c_size_t, p, ctypes.c_size_t,
                                 p, p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_int, p, ctypes.c_int, p]
    args = lambda N, ta=0, tb=0, tc=0, ct=0, k=8, opa=0, fast=1: (None, opa, 0, 8, 8, k, ta, tb, tc, None, None, 8,
                                                                  None, k, None, None, 8, N, fast, None, ct, None)
    assert lib.gemmul8_gemm(*args(1)) == -1
    assert lib.gemmul8_gemm(*args(21)) == -1
    assert lib.gemmul8_gemm(*args(14, ta=2)) == -2          # complex A with real B
    assert lib.gemmul8_gemm(*args(14, ta=2, tb=2, tc=2)) == -2  # complex types need COMPLEX_BIG_MATRIX_ENCODE
    assert lib.gemmul8_gemm(*args(14, ta=2, tb=2, tc=2, ct=1, opa=3, fast=0)) == -3  # op out of range
    assert lib.gemmul8_gemm(*args(14, k=(1 << 22) + 1)) == -4          # fast: beyond the encode grid
    assert lib.gemmul8_gemm(*args(14, k=(1 << 19) - 63, fast=0)) == -4  # accurate: int32 bound product


def test_crt_parts_errors_host_only():
    """gemmul8_crt_partial / gemmul8_crt_finish (the reduce of partial CRT sums) reject bad arguments before
    anything touches the device, with the codes include/gemmul8_c.h gives; empty outputs are a no-op"""
    lib = ctypes.CDLL(LIB)
    p, sz, u, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_int
    lib.gemmul8_crt_partial.restype = i
    lib.gemmul8_crt_partial.argtypes = [p, sz, sz, sz, u, i, i, p, u, u, p, sz]
    lib.gemmul8_crt_finish.restype = i
    lib.gemmul8_crt_finish.argtypes = [p, sz, sz, sz, u, i, i, p, p, p, sz, p, p, sz]
    part = lambda N=14, tc=0, ct=0, j0=0, j1=14, lds=8, m=8: lib.gemmul8_crt_partial(
        None, m, 8, 8, N, tc, ct, None, j0, j1, None, lds)
    fin = lambda N=14, tc=0, ct=0, lds=8, ldc=8, m=8: lib.gemmul8_crt_finish(
        None, m, 8, 8, N, tc, ct, None, None, None, ldc, None, None, lds)
    assert part(N=1) == -1 and part(N=21) == -1 and fin(N=1) == -1
    assert part(ct=1) == fin(ct=1) == -5           # complex: unsupported (real outputs only)
    assert part(tc=2) == fin(tc=2) == -2           # complex C
    assert part(lds=7) == fin(lds=7) == -4         # lds < m
    assert fin(ldc=7) == -4
    assert part(j0=3, j1=2) == -1 and part(j1=15) == -1  # moduli range
    assert part(m=0, lds=0) == 0 and fin(m=0, lds=0, ldc=0) == 0


def test_complex_karatsuba_layout():
    """complex compute types run Karatsuba sub-products (3 per modulus, csrc/oz2_common.hpp); the
    workspace also holds the accurate-mode big-matrix bound plane; real layouts are unchanged"""
    if os.environ.get("GEMMUL8_CPLX_PRODUCTS"):
        return
    import gemmul8 as G
    # the size rule (oz2_common.hpp kara_default): Karatsuba from k >= 3072 and m >= 1024
    for m, n, k in ((70, 90, 333), (1024, 1024, 1024), (2048, 2048, 2048), (256, 4096, 4096), (8192, 8192, 1024)):
        L = G.layout(m, n, k, 12, G.COMPLEX_BIG_MATRIX_ENCODE)
        assert L["nsub"] == 1 and L["m_pad"] == L["bm_pad"] == -(-2 * m // 256) * 256 and L["ldr"] == L["m_pad"]
    for m, n, k in ((3072, 3072, 3072), (4096, 256, 4096), (4096, 4096, 4096)):
        L = G.layout(m, n, k, 12, G.COMPLEX_BIG_MATRIX_ENCODE)
        assert L["nsub"] == 3 and L["vsA"] == -(-m // 256) * 256 and L["vsB"] == -(-n // 256) * 256
        assert L["planeR"] == 3 * L["subR"] == 3 * L["vsA"] * L["vsB"] and L["ldr"] == L["vsA"]
        kb = -(-k // 64) * 64
        assert L["planeA"] == 3 * L["vsA"] * kb and L["subA"] == L["vsA"] * kb and L["subB"] == L["vsB"] * kb
        assert L["offB"] - L["offA"] >= max(12 * L["planeA"], L["bm_pad"] * 2 * kb)
        assert L["offR"] - L["offB"] >= max(12 * L["planeB"], -(-n // 256) * 256 * 2 * kb)
        assert L["bm_pad"] == -(-2 * m // 256) * 256
        assert G.workSize(m, n, k, 12, G.COMPLEX_BIG_MATRIX_ENCODE) == L["total"]
        R = G.layout(m, n, k, 12, G.REAL_DEFAULT)
        assert R["nsub"] == 1 and R["ldr"] == R["m_pad"] and R["planeR"] == R["m_pad"] * R["n_pad"]


def test_interposer_exports_and_has_no_runtime_dependency():
    """libgemmul8_hijack.so: the intercepted hipBLAS / rocBLAS GEMM symbols, and no link-time HIP
    or BLAS dependency (a second HIP runtime in a framework process would break it)."""
    import subprocess
    so = os.path.join(os.path.dirname(LIB), "libgemmul8_hijack.so")
    assert os.path.exists(so)
    syms = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True).stdout
    for s in ("hipblasDgemm", "hipblasZgemm", "hipblasSgemm", "hipblasCgemm", "hipblasDgemmStridedBatched",
              "hipblasZgemmStridedBatched", "rocblas_dgemm", "rocblas_zgemm", "rocblas_sgemm", "rocblas_cgemm"):
        assert f" T {s}\n" in syms, s
    needed = subprocess.run(["readelf", "-d", so], capture_output=True, text=True).stdout
    assert "amdhip64" not in needed and "hipblas" not in needed and "rocblas" not in needed
