"""Live parity against the REFERENCE's own HIP build (oracle/_ref, compiled from the unmodified
/root/reference sources by oracle/ref/Makefile) on the same device inputs, up to the full
BASELINE size (cfg2: 8192^3, 14 moduli).  Expectation: C bit-identical.

Also records both implementations' wall time per call into gpurun_out/ref_compare.json
(the reference's own 4 phase timers include its device-wide syncs)."""
import json
import os
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ref_sweep import CODES, _extreme, _ref, sweep  # noqa: E402

RESULTS = {}


# (ta, tb, tc, m, n, k, num_moduli, fast, opA, opB, computeType)
@pytest.mark.parametrize("case", [
    ("d", "d", "d", 1024, 1024, 1024, 14, 1, 0, 0, 0),
    ("d", "d", "d", 1000, 700, 1500, 8, 1, 0, 0, 0),
    ("s", "s", "s", 1024, 768, 2048, 6, 1, 0, 0, 0),
    ("d", "s", "d", 2048, 1536, 1000, 10, 0, 0, 0, 0),
    ("d", "d", "d", 1536, 1024, 2048, 14, 0, 0, 0, 0),
    ("z", "z", "z", 512, 640, 384, 12, 1, 0, 0, 1),
    ("z", "z", "z", 600, 500, 700, 12, 1, 2, 1, 1),    # complex op C x op T
    ("z", "z", "z", 250, 300, 301, 12, 0, 0, 0, 1),    # complex accurate, k mod 4 = 1 (m = 256 hits a reference defect)
    ("c", "c", "c", 512, 384, 500, 7, 0, 0, 0, 3),     # Karatsuba, accurate
    ("z", "z", "z", 250, 300, 301, 12, 0, 0, 2, 1),    # complex accurate, op N x op C
    ("z", "z", "z", 300, 300, 401, 12, 0, 2, 2, 1),    # complex accurate, op C x op C (square: DESIGN 10.12)
    ("c", "c", "c", 400, 320, 500, 7, 0, 1, 2, 3),     # Karatsuba accurate, op T x op C
    ("c", "c", "c", 300, 256, 333, 6, 1, 1, 2, 2),     # classic, op T x op C
    ("d", "d", "d", 8192, 8192, 8192, 14, 1, 0, 0, 0),   # cfg2
    ("s", "s", "s", 1024, 1024, 1024, 4, 1, 0, 0, 0),     # cfg1 shape on the GPU
    ("d", "s", "d", 8192, 8192, 8192, 10, 0, 0, 0, 0),    # cfg4
    ("z", "z", "z", 4096, 4096, 4096, 12, 1, 0, 0, 1),    # cfg5
])
def test_same_inputs_same_bits(case):
    import torch
    import gemmul8 as G
    ta, tb, tc, m, n, k, N, fast, opA, opB, ct = case
    lib = _ref()
    tdt = {"d": torch.float64, "s": torch.float32, "z": torch.complex128, "c": torch.complex64}
    A = G.randmat(k, m, tdt[ta], 0.5, 123456) if opA else G.randmat(m, k, tdt[ta], 0.5, 123456)
    B = G.randmat(n, k, tdt[tb], 0.5, 654321) if opB else G.randmat(k, n, tdt[tb], 0.5, 123456)
    lda, ldb = (k if opA else m), (n if opB else k)
    C_ref = torch.zeros((n, m), dtype=tdt[tc], device="cuda")
    C_new = torch.zeros_like(C_ref)
    npt = {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}[tc]
    one, zero = np.array([1], npt), np.array([0], npt)
    wref = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + 16 * A.numel() + (1 << 20), dtype=torch.uint8,
                       device="cuda")
    wnew = G.alloc_work(m, n, k, N, ct)

    def run_ref():
        rc = lib.ref_gemm(CODES[ta], CODES[tb], CODES[tc], opA, opB, m, n, k, one.ctypes.data, A.data_ptr(), lda,
                          B.data_ptr(), ldb, zero.ctypes.data, C_ref.data_ptr(), m, N, fast, ct, wref.data_ptr(), None)
        assert rc == 0

    def run_new():
        G.gemm(opA, opB, m, n, k, 1.0, A, lda, B, ldb, 0.0, C_new, m, N, bool(fast), wnew, ct)

    run_ref()
    run_new()
    torch.cuda.synchronize()
    same = torch.equal(C_ref, C_new)
    nbad = int((C_ref != C_new).sum().item())
    # timing (median of a few calls each, after the warm-up above)
    tt = {}
    for name, fn in (("reference", run_ref), ("mi355x", run_new)):
        ts = []
        for _ in range(3 if m * n * k > 1e11 else 5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        tt[name] = float(np.median(ts))
    mult = 8 if ct else 2
    RESULTS["%s%s%s_%dx%dx%d_N%d_%s_op%d%d_ct%d" % (ta, tb, tc, m, n, k, N, "fast" if fast else "accu", opA, opB,
                                                   ct)] = {
        "bit_identical": bool(nbad == 0), "n_diff": nbad,
        "ref_ms": tt["reference"] * 1e3, "mi355x_ms": tt["mi355x"] * 1e3,
        "ref_tflops": mult * m * n * k / tt["reference"] / 1e12, "mi355x_tflops": mult * m * n * k / tt["mi355x"] / 1e12}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ref_compare.json"), "w") as f:
        json.dump(RESULTS, f, indent=1)
    assert same and nbad == 0, f"{nbad} elements differ from the reference"


# (ta, tb, tc, m, n, k, num_moduli, fast, computeType)
@pytest.mark.parametrize("case", [
    ("d", "d", "d", 300, 260, 500, 14, 1, 0),
    ("d", "d", "d", 300, 260, 500, 14, 0, 0),
    ("d", "d", "d", 300, 260, 500, 20, 1, 0),
    ("s", "s", "s", 200, 190, 300, 8, 1, 0),
    ("s", "s", "s", 200, 190, 300, 8, 0, 0),
    ("d", "s", "d", 200, 190, 300, 12, 1, 0),
    ("z", "z", "z", 160, 150, 200, 12, 1, 1),
    ("z", "z", "z", 160, 150, 200, 12, 0, 1),
    ("c", "c", "c", 160, 150, 200, 7, 0, 3),    # Karatsuba (complex double only up to 7 moduli: DESIGN 10.5)
    ("z", "z", "z", 160, 150, 200, 6, 1, 2),    # classic
])
def test_extreme_magnitudes_same_bits(case):
    """Subnormal, zero, single-element and overflowing-norm rows of A and columns of B: the shifts the
    reference derives from them (log2 of round-up sums that under- or overflow, ilogb of subnormals)
    and everything after them give the same C bits, NaN / Inf included, as the reference's own build."""
    import torch
    import gemmul8 as G
    ta, tb, tc, m, n, k, N, fast, ct = case
    lib = _ref()
    tdt = {"d": torch.float64, "s": torch.float32, "z": torch.complex128, "c": torch.complex64}
    dbl = {"d": True, "s": False, "z": True, "c": False}
    A = G.randmat(m, k, tdt[ta], 0.5, 123456)  # (k, m) tensor: A[e, v] = element e of row v
    B = G.randmat(k, n, tdt[tb], 0.5, 654321)  # (n, k) tensor: B[v, e] = element e of column v
    ext = lambda d: (1e200, 1e-200, 1e-310) if dbl[d] else (1e25, 1e-25, 1e-40)
    _extreme(A, 1, *ext(ta))
    _extreme(B, 0, *ext(tb))
    C_ref = torch.zeros((n, m), dtype=tdt[tc], device="cuda")
    C_new = torch.zeros_like(C_ref)
    npt = {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}[tc]
    one, zero = np.array([1], npt), np.array([0], npt)
    wref = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + 16 * A.numel() + (1 << 20), dtype=torch.uint8,
                       device="cuda")
    rc = lib.ref_gemm(CODES[ta], CODES[tb], CODES[tc], 0, 0, m, n, k, one.ctypes.data, A.data_ptr(), m,
                      B.data_ptr(), k, zero.ctypes.data, C_ref.data_ptr(), m, N, fast, ct, wref.data_ptr(), None)
    assert rc == 0
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C_new, m, N, bool(fast), G.alloc_work(m, n, k, N, ct), ct)
    torch.cuda.synchronize()
    a = C_ref.view(torch.uint8).cpu().numpy()
    b = C_new.view(torch.uint8).cpu().numpy()
    nbad = int((a != b).sum())
    assert nbad == 0, f"{nbad} bytes differ from the reference"
    # the inputs did reach the interesting regimes: the normal part of C is finite and nonzero
    assert torch.isfinite(C_new[6:, 6:]).all() and (C_new[6:, 6:] != 0).any()


# (ta, tb, tc, num_moduli, fast, computeType, opA, opB)
@pytest.mark.parametrize("case", [
    ("d", "d", "d", 14, 1, 0, 0, 0), ("d", "d", "d", 14, 0, 0, 0, 0), ("s", "s", "s", 8, 1, 0, 0, 0),
    ("z", "z", "z", 12, 1, 1, 0, 0), ("c", "c", "c", 7, 0, 3, 0, 0),
    ("d", "d", "d", 14, 0, 0, 1, 1), ("d", "s", "d", 12, 0, 0, 0, 0), ("s", "d", "s", 8, 0, 0, 1, 0),
    ("z", "z", "z", 12, 0, 1, 0, 0), ("z", "z", "z", 6, 0, 2, 0, 2), ("c", "c", "c", 7, 1, 3, 1, 0),
])
def test_nonfinite_inputs_same_bits(case):
    """A NaN in one row of A, +Inf in one column of B and -Inf in another: C matches the reference's
    build byte for byte, whatever the non-finite shifts make of the affected rows and columns."""
    import torch
    import gemmul8 as G
    ta, tb, tc, N, fast, ct, opA, opB = case
    m, n, k = 130, 120, 140
    lib = _ref()
    tdt = {"d": torch.float64, "s": torch.float32, "z": torch.complex128, "c": torch.complex64}
    # stored column-major: op N A is m x k (tensor (k, m)), op T A is k x m (tensor (m, k)); likewise B
    A = G.randmat(k, m, tdt[ta], 0.5, 123456) if opA else G.randmat(m, k, tdt[ta], 0.5, 123456)
    B = G.randmat(n, k, tdt[tb], 0.5, 654321) if opB else G.randmat(k, n, tdt[tb], 0.5, 654321)
    A[7, 5] = float("nan")
    B[9, 3] = float("inf")
    B[11, 100] = -float("inf")
    lda, ldb = (k if opA else m), (n if opB else k)
    C_ref = torch.zeros((n, m), dtype=tdt[tc], device="cuda")
    C_new = torch.zeros_like(C_ref)
    npt = {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}[tc]
    one, zero = np.array([1], npt), np.array([0], npt)
    wref = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + 16 * A.numel() + (1 << 20), dtype=torch.uint8,
                       device="cuda")
    rc = lib.ref_gemm(CODES[ta], CODES[tb], CODES[tc], opA, opB, m, n, k, one.ctypes.data, A.data_ptr(), lda,
                      B.data_ptr(), ldb, zero.ctypes.data, C_ref.data_ptr(), m, N, fast, ct, wref.data_ptr(), None)
    assert rc == 0
    G.gemm(opA, opB, m, n, k, 1.0, A, lda, B, ldb, 0.0, C_new, m, N, bool(fast), G.alloc_work(m, n, k, N, ct), ct)
    torch.cuda.synchronize()
    nbad = int((C_ref.view(torch.uint8) != C_new.view(torch.uint8)).sum())
    assert nbad == 0, f"{nbad} bytes differ from the reference"


# (type, num_moduli, computeType, alpha, beta, non-finite Im(C))
@pytest.mark.parametrize("case", [
    ("z", 6, 1, 1.5 - 0.5j, 0.0, False), ("c", 6, 1, 1.5 - 0.5j, 0.0, False),
    ("z", 6, 1, 1.5 - 0.5j, 0.25 + 0.75j, False), ("c", 6, 1, 1.5 - 0.5j, 0.25 + 0.75j, False),
    ("z", 6, 1, 1.0 + 1.0j, 1.0, False), ("c", 6, 1, 1.0 + 1.0j, 1.0, False),
    ("c", 6, 1, 2.5, 1.0, False), ("z", 14, 1, 2.5, -0.5j, False), ("c", 8, 1, 2.5, 0.5, False),
    ("z", 14, 1, 1.5 - 0.5j, 0.0, False), ("z", 14, 1, 1.5 - 0.5j, 0.25 + 0.75j, False),
    ("z", 19, 1, 0.3 + 1.7j, -1.25 + 0.5j, False), ("c", 12, 1, 0.3 + 1.7j, -1.25 + 0.5j, False),
    ("z", 6, 1, 1.0, 1.0, True), ("c", 6, 1, 2.0, 0.5, True), ("z", 6, 1, 2.5, 1.0, True),
    ("z", 6, 1, 1.5 - 0.5j, 0.25 + 0.75j, True), ("c", 7, 3, 1.0, 0.0, True), ("z", 6, 2, 1.0, 0.0, True),
])
def test_complex_alpha_beta_same_bits(case):
    """Complex and general alpha / beta through the reference's epilogue kernels (_a1, _ab, CAdd),
    finite and with Inf / NaN in Im(C): the same bytes as the reference's build.  (alpha = 1 with
    another beta (_1b) and beta = 0 reading C are the reference's non-BLAS variants)"""
    import torch
    import gemmul8 as G
    t, N, ct, al, be, nonfinite = case
    m, n, k = 150, 130, 256
    lib = _ref()
    tdt = {"z": torch.complex128, "c": torch.complex64}[t]
    npt = {"z": np.complex128, "c": np.complex64}[t]
    A = G.randmat(m, k, tdt, 0.5, 123456)
    B = G.randmat(k, n, tdt, 0.5, 654321)
    C0 = G.randmat(m, n, tdt, 0.5, 777)
    if nonfinite:
        C0[4, 3] = complex(0.5, float("inf"))
        C0[9, 11] = complex(-0.25, float("nan"))
    C_ref, C_new = C0.clone(), C0.clone()
    alpha, beta = np.array([al], npt), np.array([be], npt)
    wref = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + (1 << 22), dtype=torch.uint8, device="cuda")
    rc = lib.ref_gemm(CODES[t], CODES[t], CODES[t], 0, 0, m, n, k, alpha.ctypes.data, A.data_ptr(), m, B.data_ptr(), k,
                      beta.ctypes.data, C_ref.data_ptr(), m, N, 1, ct, wref.data_ptr(), None)
    assert rc == 0
    G.gemm(0, 0, m, n, k, complex(al), A, m, B, k, complex(be), C_new, m, N, True, G.alloc_work(m, n, k, N, ct), ct)
    torch.cuda.synchronize()
    nbad = int((C_ref.view(torch.uint8) != C_new.view(torch.uint8)).sum())
    assert nbad == 0, f"{nbad} bytes differ from the reference"


@pytest.mark.parametrize("mode", [
    dict(seed=101, extreme=False, ab_mode="general", ld=False),
    dict(seed=102, extreme=False, ab_mode="general", ld=True),
    dict(seed=103, extreme=True, ab_mode="general", ld=False),
    dict(seed=104, extreme=True, ab_mode="general", ld=False, ref_epi=True),
])
def test_randomized_live_parity(mode):
    """tests/ref_sweep.py: 300 random calls (the 12 type combinations, N = 2..20, both modes,
    ops N/T/C, the three complex compute types, general and complex alpha / beta; padded leading dimensions;
    extreme and non-finite inputs) through both builds, C compared byte for byte.  Skipped: the input classes
    of DESIGN.md section 10; with non-finite inputs, differences confined to the rows / columns that hold them."""
    _ref()
    out = sweep(300, mode["seed"], extreme=mode["extreme"], ab_mode=mode["ab_mode"], ld=mode["ld"],
                         verbose=False, ref_epi=mode.get("ref_epi", False))
    assert out["cases"] == 300
    assert not out["failures"], out["failures"][:3]


# (type, num_moduli, alpha, beta, NaN / Inf in C): the reference's non-BLAS epilogue variants (DESIGN.md 10.3,
# 10.16), which the default BLAS mode does not reproduce: alpha = 1 with beta off {0, 1} (_1b), alpha != 1 with
# beta = 1 at two moduli levels (_2_a1), alpha != 1 with beta = 0 reading C (_ab); one- and two-level moduli
@pytest.mark.parametrize("case", [
    ("d", 6, 1.0, 0.5, False), ("d", 14, 1.0, -0.75, False), ("d", 14, 2.5, 1.0, False), ("d", 6, 2.5, 1.0, False),
    ("d", 14, 2.5, 0.0, True), ("d", 9, -1.5, 0.0, False), ("s", 8, 1.0, 0.5, False), ("s", 12, 2.5, 0.0, True),
    ("s", 10, 2.5, 1.0, False),
    ("z", 6, 1.0, 0.25 + 0.75j, False), ("z", 14, 1.0, -1.25 + 0.5j, False), ("z", 14, 1.5 - 0.5j, 1.0, False),
    ("z", 6, 1.5 - 0.5j, 1.0, False), ("z", 14, 0.3 + 1.7j, 0.0, True), ("z", 12, 2.5, 0.0, False),
    ("c", 8, 1.0, 0.25 + 0.75j, False), ("c", 12, 1.5 - 0.5j, 1.0, False), ("c", 10, 0.3 + 1.7j, 0.0, True),
])
def test_reference_epilogue_mode_same_bits(case):
    """gemmul8_set_epilogue(GEMMUL8_EPILOGUE_REFERENCE): the reference's epilogue kernels bit for bit, including
    the alpha / beta classes where they depart from BLAS; the same call in the default mode follows BLAS and
    differs there; the CPU oracle with quirks=True restates the same bits"""
    import torch
    import gemmul8 as G
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    t, N, al, be, nonfinite = case
    m, n, k = 150, 130, 256
    lib = _ref()
    cplx = t in "zc"
    ct = 1 if cplx else 0
    tdt = {"d": torch.float64, "s": torch.float32, "z": torch.complex128, "c": torch.complex64}[t]
    npt = {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}[t]
    A = G.randmat(m, k, tdt, 0.5, 123456)
    B = G.randmat(k, n, tdt, 0.5, 654321)
    C0 = G.randmat(m, n, tdt, 0.5, 777)
    if nonfinite:
        C0[4, 3] = float("inf")
        C0[9, 11] = float("nan")
        C0[2, 5] = -0.0
    C_ref, C_new, C_blas = C0.clone(), C0.clone(), C0.clone()
    alpha, beta = np.array([al], npt), np.array([be], npt)
    wref = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + (1 << 22), dtype=torch.uint8, device="cuda")
    rc = lib.ref_gemm(CODES[t], CODES[t], CODES[t], 0, 0, m, n, k, alpha.ctypes.data, A.data_ptr(), m, B.data_ptr(), k,
                      beta.ctypes.data, C_ref.data_ptr(), m, N, 1, ct, wref.data_ptr(), None)
    assert rc == 0
    a, b = (complex(al), complex(be)) if cplx else (float(al.real if isinstance(al, complex) else al), float(be))
    work = G.alloc_work(m, n, k, N, ct)
    prev = G.set_epilogue("reference")
    try:
        assert G.get_epilogue() == "reference"
        G.gemm(0, 0, m, n, k, a, A, m, B, k, b, C_new, m, N, True, work, ct)
    finally:
        G.set_epilogue(prev)
    G.gemm(0, 0, m, n, k, a, A, m, B, k, b, C_blas, m, N, True, work, ct)
    torch.cuda.synchronize()
    nbad = int((C_ref.view(torch.uint8) != C_new.view(torch.uint8)).sum())
    assert nbad == 0, f"{nbad} bytes differ from the reference in reference-epilogue mode"
    Co = np.ascontiguousarray(O.gemm(A.cpu().numpy().T, B.cpu().numpy().T, N, True, npt, al, be,
                                     C0.cpu().numpy().T, quirks=True))
    Cg = np.ascontiguousarray(C_new.cpu().numpy().T)
    diff = Co.view(np.uint8) != Cg.view(np.uint8)
    assert not diff.any(), f"oracle (quirks): {int(diff.sum())} bytes differ, first at {np.argwhere(diff)[0]}"
    numM2 = N >= 8 and t in "dz"
    departs = (al == 1 and be not in (0, 1)) or (al != 1 and be == 1 and numM2) or (al != 1 and be == 0 and nonfinite)
    if departs:
        assert not torch.equal(C_blas.view(torch.uint8), C_new.view(torch.uint8))
