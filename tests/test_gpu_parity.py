"""GPU parity: the HIP path (through the C ABI) against the CPU oracle restatement.

Bit-exact expectations (integer / exactly restated arithmetic):
  * shifts sftA/sftB (fast mode: round-up norms reduced in the reference's order;
    the only non-restated op is v_log_f32, whose effect is reported separately),
  * every int8 slice of every modulus, including zero padding,
  * every residue plane (the int8 products are exact),
  * C bit-for-bit for f64/f32/complex outputs.
"""
import os
import sys

import numpy as np
import pytest

from util import bits_equal, randmat_np, untile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

pytestmark = pytest.mark.gpu

NP2T = None


def _torch():
    import torch
    return torch


def to_dev(X):
    """column-major numpy -> device tensor holding the same column-major bytes"""
    torch = _torch()
    Xf = np.asfortranarray(X)
    return torch.from_numpy(np.ascontiguousarray(Xf.T)).cuda()


def run_gpu(A, B, N, fast=True, opA=0, opB=0, out_dtype=None, alpha=1.0, beta=0.0, C0=None, ctype=None):
    torch = _torch()
    import gemmul8 as G
    A = np.asfortranarray(A)
    B = np.asfortranarray(B)
    m = A.shape[1] if opA else A.shape[0]
    k = A.shape[0] if opA else A.shape[1]
    n = B.shape[0] if opB else B.shape[1]
    out_dtype = out_dtype or np.result_type(A.dtype, B.dtype)
    cplx = np.iscomplexobj(A)
    ct = (ctype or G.COMPLEX_BIG_MATRIX_ENCODE) if cplx else G.REAL_DEFAULT
    if C0 is None:
        C0 = np.zeros((m, n), out_dtype, order="F")
    dA, dB, dC = to_dev(A), to_dev(B), to_dev(np.asfortranarray(C0.astype(out_dtype)))
    ws = G.workSize(m, n, k, N, ct)
    work = torch.full((ws,), 0xA5, dtype=torch.uint8, device="cuda")
    G.gemm(opA, opB, m, n, k, alpha, dA, A.shape[0], dB, B.shape[0], beta, dC, m, N, fast, work, ct)
    torch.cuda.synchronize()
    C = np.asfortranarray(dC.cpu().numpy().T)
    return C, work.cpu().numpy(), G.layout(m, n, k, N, ct)


def ws_sft(wsb, L, m, n):
    sA = wsb[L["offSftA"]:L["offSftA"] + 2 * m].view(np.int16)
    sB = wsb[L["offSftB"]:L["offSftB"] + 2 * n].view(np.int16)
    return sA.copy(), sB.copy()


def ws_planes(wsb, L, N, which):
    off, plane, vpad = (L["offA"], L["planeA"], L["m_pad"]) if which == "A" else (L["offB"], L["planeB"], L["n_pad"])
    return [untile(wsb[off + j * plane: off + (j + 1) * plane].tobytes(), vpad, L["k_pad"]) for j in range(N)]


def ws_residues(wsb, L, N):
    R = wsb[L["offR"]:L["offR"] + N * L["planeR"]].reshape(N, L["n_pad"], L["m_pad"])
    return R


def check_full(A, B, N, fast=True, opA=0, opB=0, out_dtype=None, alpha=1.0, beta=0.0, C0=None, vt=None, ctype=None):
    from oracle import oracle as O
    A = np.asfortranarray(A)
    B = np.asfortranarray(B)
    m = A.shape[1] if opA else A.shape[0]
    k = A.shape[0] if opA else A.shape[1]
    n = B.shape[0] if opB else B.shape[1]
    cplx = np.iscomplexobj(A)
    out_dtype = out_dtype or np.result_type(A.dtype, B.dtype)
    C, wsb, L = run_gpu(A, B, N, fast, opA, opB, out_dtype, alpha, beta, C0, ctype)
    A8o, B8o, sAo, sBo = O.scaling(A, B, N, fast, opA, opB, vt, ctype=ctype)
    sA, sB = ws_sft(wsb, L, m, n)
    agree_A = float(np.mean(sA == sAo)) if m else 1.0
    agree_B = float(np.mean(sB == sBo)) if n else 1.0
    assert agree_A == 1.0 and agree_B == 1.0, (agree_A, agree_B, np.nonzero(sA != sAo), np.nonzero(sB != sBo))
    Co = O.gemm(A, B, N, fast, out_dtype, alpha, beta, C0, opA, opB, vt, ctype=ctype)
    if L["nsub"] == 3:  # Karatsuba complex products: planes derived from the oracle's big matrix
        check_kara_planes(wsb, L, N, m, n, k, A8o, B8o)
        assert bits_equal(C, Co), f"C mismatch: max |diff| {np.max(np.abs(C - Co))}"
        return C, Co
    # slices (with the complex imaginary block at kblk instead of k) and zero padding
    kblk = L["kblk"]
    for which, X8o, vpad, nv in (("A", A8o, L["m_pad"], (2 * m if cplx else m)), ("B", B8o, L["n_pad"], n)):
        planes = ws_planes(wsb, L, N, which)
        for j in range(N):
            P = planes[j]
            exp = np.zeros((vpad, L["k_pad"]), np.int8)
            if cplx:
                exp[:nv, :k] = X8o[j][:, :k]
                exp[:nv, kblk:kblk + k] = X8o[j][:, k:]
            else:
                exp[:nv, :k] = X8o[j]
            assert np.array_equal(P, exp), f"{which} slice mismatch modulus {j}: {np.argwhere(P != exp)[:5]}"
    R = ws_residues(wsb, L, N)
    Ro = O.residues(A8o, B8o)
    mr = 2 * m if cplx else m
    assert np.array_equal(R[:, :n, :mr], Ro), "residue mismatch"
    assert bits_equal(C, Co), f"C mismatch: max |diff| {np.max(np.abs(C - Co))}"
    return C, Co


def _center(x, p):
    """symmetric representative of x mod p as the int8 byte the encoder stores"""
    r = np.mod(x, p)
    r = np.where(r > (p - 1) // 2, r - p, r)
    return r.astype(np.int64).astype(np.int8)


def check_kara_planes(wsb, L, N, m, n, k, A8o, B8o):
    """Karatsuba layout (csrc/oz2_common.hpp): per modulus, slice sub-blocks [re | im | re + im] of
    vsA rows / vsB columns, and residue sub-planes Ar Br, Ai Bi, (Ar + Ai)(Br + Bi) mod p.  The
    oracle's big-matrix slices hold Ar = A8[:m, :k], Ai = A8[m:, :k], Br = B8[:, :k], Bi = B8[:, k:]
    (scaling.hpp:753-838, 1150-1230); its residues Re(AB) = rows [0, m), Im(AB) = rows [m, 2m)."""
    from gen_tables import MODULI
    vsA, vsB, kp = L["vsA"], L["vsB"], L["k_pad"]
    Ro = None
    Rw = wsb[L["offR"]:L["offR"] + N * L["planeR"]].reshape(N, 3, vsB, vsA)
    for j in range(N):
        p = MODULI[j]
        Ar, Ai = A8o[j][:m, :k].astype(np.int64), A8o[j][m:2 * m, :k].astype(np.int64)
        Br, Bi = B8o[j][:, :k].astype(np.int64), B8o[j][:, k:].astype(np.int64)
        for which, (Xr, Xi), vs, off, plane in (("A", (Ar, Ai), vsA, L["offA"], L["planeA"]),
                                                ("B", (Br, Bi), vsB, L["offB"], L["planeB"])):
            P = untile(wsb[off + j * plane: off + (j + 1) * plane].tobytes(), 3 * vs, kp)
            exp = np.zeros((3 * vs, kp), np.int8)
            nv = Xr.shape[0]
            exp[:nv, :k] = Xr
            exp[vs:vs + nv, :k] = Xi
            exp[2 * vs:2 * vs + nv, :k] = _center(Xr + Xi, p)
            assert np.array_equal(P, exp), f"{which} Karatsuba slice mismatch modulus {j}: {np.argwhere(P != exp)[:5]}"
        S_A, S_B = _center(Ar + Ai, p).astype(np.int64), _center(Br + Bi, p).astype(np.int64)
        for s, (X, Y) in enumerate(((Ar, Br), (Ai, Bi), (S_A, S_B))):
            exp = np.mod(Y @ X.T, p).astype(np.uint8)  # [col][row]
            got = Rw[j, s, :n, :m]
            assert np.array_equal(got, exp), f"Karatsuba residue mismatch modulus {j} sub-product {s}"
        if Ro is None:
            Ro = O_residues(A8o, B8o)
        re = np.mod(Rw[j, 0, :n, :m].astype(np.int64) - Rw[j, 1, :n, :m], p)
        im = np.mod(Rw[j, 2, :n, :m].astype(np.int64) - Rw[j, 0, :n, :m] - Rw[j, 1, :n, :m], p)
        assert np.array_equal(re, Ro[j][:, :m]) and np.array_equal(im, Ro[j][:, m:2 * m]), f"Re/Im residues modulus {j}"


def O_residues(A8o, B8o):
    from oracle import oracle as O
    return O.residues(A8o, B8o)


@pytest.mark.parametrize("m,n,k", [(16, 16, 16), (33, 47, 100), (256, 256, 256), (300, 260, 513), (1, 1, 1)])
@pytest.mark.parametrize("N", [2, 7, 8, 14, 20])
def test_dgemm_fast(m, n, k, N):
    rng = np.random.default_rng(1000 * m + n + k + N)
    check_full(randmat_np(rng, m, k), randmat_np(rng, k, n), N)


@pytest.mark.parametrize("N", [4, 8, 13, 19])
def test_sgemm_fast(N):
    rng = np.random.default_rng(N)
    check_full(randmat_np(rng, 130, 77, dtype=np.float32), randmat_np(rng, 77, 90, dtype=np.float32), N)


@pytest.mark.parametrize("N", [8, 10, 14])
def test_mixed_accurate(N):
    rng = np.random.default_rng(7 + N)
    A = randmat_np(rng, 200, 150)
    B = randmat_np(rng, 150, 120, dtype=np.float32)
    check_full(A, B, N, fast=False)
    check_full(B.T.copy().astype(np.float32), A.T.copy(), N, fast=False)


@pytest.mark.parametrize("m,n,k,N,tb,opB", [
    (700, 1400, 16000, 10, np.float32, 0),   # the cfg4 form (f64 x f32), ragged last column tile
    (512, 2048, 16384, 12, np.float64, 0),
    (600, 1300, 16000, 8, np.float64, 1),    # op(B) = T: strided columns
    (300, 600, 40000, 14, np.float64, 0),
])
def test_accurate_two_streams(m, n, k, N, tb, opB):
    """Accurate mode at (m + n) k >= 2^25, where operand B's passes run on the second stream (the lane):
    shifts, every slice, residues and C against the oracle, long k, ragged column tiles."""
    rng = np.random.default_rng(m + n + k)
    A = randmat_np(rng, m, k)
    B = randmat_np(rng, k, n, dtype=tb)
    if opB:
        B = np.asfortranarray(B.T)
    check_full(A, B, N, fast=False, opB=opB)


@pytest.mark.parametrize("N", [6, 12])
def test_zgemm_bigmatrix(N):
    rng = np.random.default_rng(55 + N)
    check_full(randmat_np(rng, 70, 90, dtype=np.complex128), randmat_np(rng, 90, 60, dtype=np.complex128), N)


def test_cgemm_mixed_complex():
    rng = np.random.default_rng(3)
    check_full(randmat_np(rng, 40, 50, dtype=np.complex64), randmat_np(rng, 50, 30, dtype=np.complex128), 9,
               out_dtype=np.complex128)


@pytest.mark.parametrize("opA,opB", [(0, 1), (1, 0), (1, 1)])
def test_transposes(opA, opB):
    rng = np.random.default_rng(11)
    m, n, k = 90, 70, 110
    A = randmat_np(rng, k, m) if opA else randmat_np(rng, m, k)
    B = randmat_np(rng, n, k) if opB else randmat_np(rng, k, n)
    check_full(A, B, 14, opA=opA, opB=opB)
    check_full(A, B, 10, fast=False, opA=opA, opB=opB)


@pytest.mark.parametrize("alpha,beta", [(1.0, 1.0), (2.5, 0.0), (1.0, -0.5), (-1.5, 1.0), (0.75, 2.0)])
def test_alpha_beta(alpha, beta):
    rng = np.random.default_rng(21)
    A, B = randmat_np(rng, 64, 80), randmat_np(rng, 80, 48)
    C0 = randmat_np(rng, 64, 48)
    check_full(A, B, 14, alpha=alpha, beta=beta, C0=C0)
    check_full(A.astype(np.float32), B.astype(np.float32), 8, alpha=alpha, beta=beta, C0=C0.astype(np.float32))


TYPE_COMBOS = [  # the 12 reference specializations (gemmul8.hpp:49-287)
    ("d", "d", "d"), ("s", "s", "s"), ("d", "s", "d"), ("s", "d", "d"), ("d", "s", "s"), ("s", "d", "s"),
    ("c", "c", "c"), ("z", "z", "z"), ("z", "c", "z"), ("c", "z", "z"), ("z", "c", "c"), ("c", "z", "c"),
]
_NPT = {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}


@pytest.mark.parametrize("ta,tb,tc", TYPE_COMBOS)
def test_every_specialization(ta, tb, tc):
    rng = np.random.default_rng(len(ta + tb + tc) + ord(ta) * 7 + ord(tb) * 3 + ord(tc))
    A = randmat_np(rng, 70, 90, dtype=_NPT[ta])
    B = randmat_np(rng, 90, 50, dtype=_NPT[tb])
    check_full(A, B, 9, out_dtype=_NPT[tc])


@pytest.mark.parametrize("m,n,k,N", [(64, 40, 5000, 14), (513, 3, 70, 8), (3, 600, 129, 20), (256, 256, 64, 2)])
def test_extreme_shapes(m, n, k, N):
    rng = np.random.default_rng(m + n + k)
    check_full(randmat_np(rng, m, k), randmat_np(rng, k, n), N)


@pytest.mark.parametrize("opA,opB", [(1, 0), (2, 0), (0, 1), (0, 2), (1, 2), (2, 1), (2, 2)])
def test_complex_ops(opA, opB):
    """complex op T / op C on either side (big-matrix encode, fast mode; scaling.hpp:3736-3804)"""
    rng = np.random.default_rng(31 + 3 * opA + opB)
    m, n, k = 45, 38, 70
    A = randmat_np(rng, k, m, dtype=np.complex128) if opA else randmat_np(rng, m, k, dtype=np.complex128)
    B = randmat_np(rng, n, k, dtype=np.complex128) if opB else randmat_np(rng, k, n, dtype=np.complex128)
    check_full(A, B, 12, opA=opA, opB=opB)
    check_full(A.astype(np.complex64), B.astype(np.complex64), 7, opA=opA, opB=opB)


@pytest.mark.parametrize("ctype", [1, 2, 3])
@pytest.mark.parametrize("dt,N,k", [(np.complex128, 12, 45), (np.complex64, 7, 33), (np.complex128, 9, 64)])
def test_complex_accurate(ctype, dt, N, k):
    """complex accurate mode (op N), all three compute types; k mod 4 != 0 exercises the
    big-matrix B tail defect the reference's shifts carry (scaling.hpp:2313-2321)"""
    rng = np.random.default_rng(ctype * 100 + N + k)
    A, B = randmat_np(rng, 50, k, dtype=dt), randmat_np(rng, k, 36, dtype=dt)
    check_full(A, B, N, fast=False, ctype=ctype)


@pytest.mark.parametrize("ctype", [1, 2, 3])
@pytest.mark.parametrize("opA,opB", [(1, 0), (2, 0), (0, 1), (0, 2), (1, 2), (2, 1), (2, 2), (1, 1)])
def test_complex_accurate_ops(ctype, opA, opB):
    """complex accurate mode with op T / op C: shifts, slices, residues and C
    against the oracle; k mod 4 = 2 and 3 cover the tail handling of every extraction"""
    rng = np.random.default_rng(300 + 30 * ctype + 3 * opA + opB)
    for dt, m, n, k, N in ((np.complex128, 41, 35, 62, 12), (np.complex64, 30, 30, 47, 7)):
        A = randmat_np(rng, k, m, dtype=dt) if opA else randmat_np(rng, m, k, dtype=dt)
        B = randmat_np(rng, n, k, dtype=dt) if opB else randmat_np(rng, k, n, dtype=dt)
        check_full(A, B, N, fast=False, opA=opA, opB=opB, ctype=ctype)


@pytest.mark.parametrize("ctype", [2, 3])
def test_classic_karatsuba_fast(ctype):
    rng = np.random.default_rng(77 + ctype)
    A, B = randmat_np(rng, 60, 50, dtype=np.complex128), randmat_np(rng, 50, 40, dtype=np.complex128)
    check_full(A, B, 14, ctype=ctype, opA=0, opB=0)
    check_full(A.astype(np.complex64), B, 8, ctype=ctype, out_dtype=np.complex128)


def test_zero_rows_and_cols():
    rng = np.random.default_rng(5)
    A, B = randmat_np(rng, 50, 60), randmat_np(rng, 60, 40)
    A[3, :] = 0
    B[:, 7] = 0
    C, _ = check_full(A, B, 14)
    assert np.all(C[3, :] == 0) and np.all(C[:, 7] == 0)


def test_mfma_raw_product():
    """v_mfma_i32_32x32x32_i8 tile/epilogue mapping: exact int32 product of random int8 planes."""
    torch = _torch()
    import gemmul8 as G
    from util import tile
    rng = np.random.default_rng(9)
    m, n, k, N = 300, 520, 200, 2
    L = G.layout(m, n, k, N)
    A8 = np.zeros((L["m_pad"], L["k_pad"]), np.int8)
    B8 = np.zeros((L["n_pad"], L["k_pad"]), np.int8)
    A8[:m, :k] = rng.integers(-128, 128, (m, k))
    B8[:n, :k] = rng.integers(-128, 128, (n, k))
    ws = np.zeros(L["total"], np.uint8)
    ws[L["offA"]:L["offA"] + L["planeA"]] = tile(A8, L["m_pad"], L["k_pad"]).view(np.uint8)
    ws[L["offB"]:L["offB"] + L["planeB"]] = tile(B8, L["n_pad"], L["k_pad"]).view(np.uint8)
    work = torch.from_numpy(ws).cuda()
    C32 = torch.zeros((L["n_pad"], L["m_pad"]), dtype=torch.int32, device="cuda")
    import ctypes
    rc = G.lib.gemmul8_i8_product_raw(G._stream(), m, n, k, N, 0, ctypes.c_void_p(work.data_ptr()),
                                      ctypes.c_void_p(C32.data_ptr()))
    assert rc == 0
    torch.cuda.synchronize()
    got = C32.cpu().numpy().T  # (m_pad, n_pad)
    exp = A8.astype(np.int64) @ B8.astype(np.int64).T
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("fast", [True, False])
def test_flat_address_dma_path(fast, monkeypatch):
    """the product kernel's 64-bit flat LDS-DMA path (taken for slice planes of 4 GiB and more)
    forced at small sizes: same slices, residues and C as the oracle"""
    monkeypatch.setenv("GEMMUL8_FORCE_FLAT_DMA", "1")
    rng = np.random.default_rng(61 + fast)
    check_full(randmat_np(rng, 300, 513), randmat_np(rng, 513, 260), 14, fast=fast)
    check_full(randmat_np(rng, 45, 70, dtype=np.complex128), randmat_np(rng, 70, 38, dtype=np.complex128), 12,
               fast=fast)


@pytest.mark.parametrize("fast", [True, False])
def test_empty_k(fast):
    """k = 0: every residue is 0, so C = beta * C (alpha * 0 + beta * C)"""
    rng = np.random.default_rng(71)
    A = np.zeros((40, 0), np.float64, order="F")
    B = np.zeros((0, 30), np.float64, order="F")
    C0 = randmat_np(rng, 40, 30)
    C, _, _ = run_gpu(A, B, 14, fast=fast, alpha=2.0, beta=-0.5, C0=C0)
    assert np.array_equal(C, -0.5 * C0)


@pytest.mark.parametrize("fast", [True, False])
def test_long_k_signed_residue_path(fast):
    """k_pad > 2^16: the int32 products may exceed 2^30, so the epilogue takes the reference's
    signed Barrett reduction (conv_32i_2_8u.hpp:7-71) instead of the biased one"""
    rng = np.random.default_rng(72 + fast)
    check_full(randmat_np(rng, 20, 70000), randmat_np(rng, 70000, 24), 14, fast=fast)
    check_full(randmat_np(rng, 12, 40000, dtype=np.complex128), randmat_np(rng, 40000, 10, dtype=np.complex128), 12,
               fast=fast)


def test_k_beyond_int32_range_chunked():
    """padded k > 2^17, where the reference's int32 products wrap: the residue product runs in
    k-chunks of 2^16 whose residues add mod p (gemm_i8.hip), equal to the exact int64 residues of
    the oracle (oz2o_residues); real and complex, fast mode"""
    rng = np.random.default_rng(77)
    check_full(randmat_np(rng, 9, 140000), randmat_np(rng, 140000, 7), 14)
    check_full(randmat_np(rng, 5, 70000, dtype=np.complex128), randmat_np(rng, 70000, 6, dtype=np.complex128), 12)


def test_k_at_the_largest_accepted_size():
    """the largest k a call accepts (padded k of the int8 product = 2^22, fast mode): the strided encode's
    grid then has 65536 k-tiles in y, the device's limit (hipDeviceAttributeMaxGridDimY); real (k = 2^22)
    and complex (k = 2^21: the big-matrix product's k is 2^22, the complex encode's k-tiles are 32 wide);
    64 k-chunks of the residue product; and one more k-step is rejected before anything is launched"""
    import torch
    import gemmul8 as G
    rng = np.random.default_rng(3)
    check_full(randmat_np(rng, 3, 1 << 22), randmat_np(rng, 1 << 22, 5), 2)
    check_full(randmat_np(rng, 2, 1 << 21, dtype=np.complex128), randmat_np(rng, 1 << 21, 3, dtype=np.complex128), 2,
               ctype=1)
    k = (1 << 22) + 1
    A = torch.zeros((k, 3), dtype=torch.float64, device="cuda")
    B = torch.zeros((5, k), dtype=torch.float64, device="cuda")
    C = torch.zeros((5, 3), dtype=torch.float64, device="cuda")
    W = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    with pytest.raises(G.Gemmul8Error):
        G.gemm(0, 0, 3, 5, k, 1.0, A, 3, B, k, 0.0, C, 3, 2, True, W)


@pytest.mark.parametrize("fast", [True, False])
def test_more_contiguous_vectors_than_grid_rows(fast):
    """B with more than 4 Mi columns (op N: contiguous vectors; their 64-vector tiles exceed the grid's
    y limit of 65536 in the k-first encode order, so the encode walks them in x): C against the oracle,
    bit for bit (k = 64, 2 moduli; fast mode takes the one-launch pair encode, accurate mode the
    per-operand encodes and the bound product).  The reference launches its column kernel with n
    blocks in x (scaling.hpp:3731-3733)."""
    import torch
    import gemmul8 as G
    from oracle import oracle as O
    m, n, k, N = 3, (1 << 22) + 200, 64, 2
    rng = np.random.default_rng(11)
    A = randmat_np(rng, m, k)
    B = randmat_np(rng, k, n)
    dA = torch.from_numpy(np.ascontiguousarray(A.T)).cuda()
    dB = torch.from_numpy(np.ascontiguousarray(B.T)).cuda()
    dC = torch.zeros((n, m), dtype=torch.float64, device="cuda")
    W = G.alloc_work(m, n, k, N)
    G.gemm(0, 0, m, n, k, 1.0, dA, m, dB, k, 0.0, dC, m, N, fast, W)
    torch.cuda.synchronize()
    Co = np.asfortranarray(O.gemm(A, B, N, fast))
    assert np.asfortranarray(dC.cpu().numpy().T).tobytes() == Co.tobytes()


@pytest.mark.parametrize("fast", [True, False])
def test_k_chunks_forced(fast):
    """the chunked product forced at small k (GEMMUL8_KCHUNK: chunks of 2 k-steps in a child
    process) gives the same bits as one pass"""
    import os
    import subprocess
    import sys
    code = ("import sys, numpy as np; sys.path[:0] = sys.argv[1:4]\n"
            "from test_gpu_parity import check_full\nfrom util import randmat_np\n"
            "rng = np.random.default_rng(5)\n"
            f"check_full(randmat_np(rng, 300, 700), randmat_np(rng, 700, 260), 14, fast={fast})\n"
            f"check_full(randmat_np(rng, 70, 333, dtype=np.complex128), randmat_np(rng, 333, 90, dtype=np.complex128), 9, fast={fast})\n"
            "print('OK')")
    tdir = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(tdir)
    env = dict(os.environ, GEMMUL8_KCHUNK="2")
    r = subprocess.run([sys.executable, "-c", code, tdir, root, os.path.join(root, "mixed-gemmul8_amd")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-3000:]


@pytest.mark.parametrize("m,n,k,opA,opB", [(70, 90, 1100, 0, 0), (33, 130, 1536, 1, 1), (129, 40, 2048, 0, 1),
                                           (300, 7, 1500, 1, 0), (5, 64, 1024, 0, 0)])
def test_fused_split_long_k(m, n, k, opA, opB):
    """fast mode, one stream, k in (1024, 2048] and at 1024: the one-launch split (split_fused_kernel, 1536- and
    2048-element panels) for every operand form (strided / contiguous vectors): shifts, slices, residues and C
    against the oracle, with an all-zero row of op(A) and column of op(B) among the vectors"""
    rng = np.random.default_rng(m + n + k + opA + opB)
    A = randmat_np(rng, k, m) if opA else randmat_np(rng, m, k)
    B = randmat_np(rng, n, k) if opB else randmat_np(rng, k, n)
    if m > 3 and n > 3:
        (A[:, 1] if opA else A[1, :])[:] = 0.0
        (B[2, :] if opB else B[:, 2])[:] = 0.0
    check_full(A, B, 14, opA=opA, opB=opB)


@pytest.mark.parametrize("m,n,k,opA,opB", [(64, 4096, 8192, 0, 0), (4100, 48, 8000, 1, 1), (3000, 2000, 4100, 1, 0)])
def test_large_split_forms(m, n, k, opA, opB):
    """fast mode at (m + n) k >= 2^25, 2048 < k <= 8192: A op N x B op N through the pair kernels, the other forms
    with the operands on two streams (per-operand stats pass + encode).  Shifts and every slice against the
    oracle (the products and the CRT downstream are the ones the other tests check)."""
    from oracle import oracle as O
    rng = np.random.default_rng(m + n + k)
    A = randmat_np(rng, k, m) if opA else randmat_np(rng, m, k)
    B = randmat_np(rng, n, k) if opB else randmat_np(rng, k, n)
    N = 14
    _, wsb, L = run_gpu(A, B, N, True, opA, opB)
    A8o, B8o, sAo, sBo = O.scaling(np.asfortranarray(A), np.asfortranarray(B), N, True, opA, opB)
    sA, sB = ws_sft(wsb, L, m, n)
    assert np.array_equal(sA, sAo) and np.array_equal(sB, sBo)
    for which, X8o, vpad, nv in (("A", A8o, L["m_pad"], m), ("B", B8o, L["n_pad"], n)):
        planes = ws_planes(wsb, L, N, which)
        for j in range(N):
            exp = np.zeros((vpad, L["k_pad"]), np.int8)
            exp[:nv, :k] = X8o[j]
            assert np.array_equal(planes[j], exp), f"{which} slice mismatch modulus {j}"


@pytest.mark.parametrize("env", [{"GEMMUL8_FUSED_V": "8"}, {"GEMMUL8_FUSED_SPLIT": "0"}])
def test_fused_split_variants(env):
    """the one-launch split with 8 vectors per block and the two-launch split (child processes): the same
    shifts, slices and C as the oracle at k = 1024, 1536 and 2048"""
    import subprocess
    code = ("import sys, numpy as np; sys.path[:0] = sys.argv[1:4]\n"
            "from test_gpu_parity import check_full\nfrom util import randmat_np\n"
            "rng = np.random.default_rng(9)\n"
            "check_full(randmat_np(rng, 70, 1024), randmat_np(rng, 1024, 90), 14)\n"
            "check_full(randmat_np(rng, 1536, 33), randmat_np(rng, 130, 1536), 14, opA=1, opB=1)\n"
            "check_full(randmat_np(rng, 129, 2000), randmat_np(rng, 40, 2000), 8, opB=1)\n"
            "print('OK')")
    tdir = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(tdir)
    r = subprocess.run([sys.executable, "-c", code, tdir, root, os.path.join(root, "mixed-gemmul8_amd")],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-3000:]


def test_complex_karatsuba_products_forced():
    """GEMMUL8_CPLX_PRODUCTS=karatsuba (child process): complex products as Karatsuba sub-products
    at shapes where the size rule keeps the big matrix; Karatsuba slices, the three residue
    sub-planes and C against the oracle, fast and accurate (big-matrix bound), all three compute
    types, ops N/T/C, N = 20, f32 operands, low-memory mode and chunked k"""
    import subprocess
    code = ("import sys, numpy as np; sys.path[:0] = sys.argv[1:4]\n"
            "from test_gpu_parity import check_full\nfrom util import randmat_np\n"
            "import gemmul8 as G\n"
            "rng = np.random.default_rng(11)\n"
            "L = G.layout(70, 90, 333, 9, G.COMPLEX_BIG_MATRIX_ENCODE)\n"
            "assert L['nsub'] == 3, L\n"
            "for ct in (1, 2, 3):\n"
            "    check_full(randmat_np(rng, 70, 333, dtype=np.complex128), randmat_np(rng, 333, 90, dtype=np.complex128), 12, ctype=ct)\n"
            "    check_full(randmat_np(rng, 41, 62, dtype=np.complex128), randmat_np(rng, 62, 35, dtype=np.complex128), 12, fast=False, ctype=ct)\n"
            "check_full(randmat_np(rng, 50, 33, dtype=np.complex64), randmat_np(rng, 40, 50, dtype=np.complex64), 7, opA=2, opB=1)\n"
            "check_full(randmat_np(rng, 33, 50, dtype=np.complex128), randmat_np(rng, 40, 50, dtype=np.complex128), 12, opB=2)\n"
            "check_full(randmat_np(rng, 30, 47, dtype=np.complex64), randmat_np(rng, 47, 30, dtype=np.complex64), 7, fast=False, opA=2, opB=0)\n"
            "check_full(randmat_np(rng, 300, 260, dtype=np.complex128), randmat_np(rng, 260, 513, dtype=np.complex128), 20)\n"
            "check_full(randmat_np(rng, 40, 50, dtype=np.complex64), randmat_np(rng, 50, 30, dtype=np.complex128), 9, out_dtype=np.complex128)\n"
            "check_full(randmat_np(rng, 45, 70, dtype=np.complex64), randmat_np(rng, 70, 38, dtype=np.complex64), 16)\n"
            "check_full(randmat_np(rng, 5, 70000, dtype=np.complex128), randmat_np(rng, 70000, 6, dtype=np.complex128), 12)\n"
            "import torch\n"
            "m, n, k, N = 300, 260, 513, 14\n"
            "A = torch.randn((k, m), dtype=torch.complex128, device='cuda'); B = torch.randn((n, k), dtype=torch.complex128, device='cuda')\n"
            "Cs = []\n"
            "for S in (None, 2, 5):\n"
            "    W = G.alloc_work(m, n, k, N, 1, slice_planes=S); C = torch.empty((n, m), dtype=torch.complex128, device='cuda')\n"
            "    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, True, W, 1, slice_planes=S); Cs.append(C.cpu())\n"
            "assert all(torch.equal(Cs[0].view(torch.float64), c.view(torch.float64)) for c in Cs[1:])\n"
            "print('OK')")
    tdir = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(tdir)
    env = dict(os.environ, GEMMUL8_CPLX_PRODUCTS="karatsuba")
    r = subprocess.run([sys.executable, "-c", code, tdir, root, os.path.join(root, "mixed-gemmul8_amd")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-3000:]


@pytest.mark.parametrize("fast", [True, False])
def test_padded_leading_dimensions(fast):
    """lda > m, ldb > k, ldc > m (odd, so C columns are not 16-byte aligned): same bits as the
    tight layout, and C's padding rows are left untouched"""
    torch = _torch()
    import gemmul8 as G
    rng = np.random.default_rng(81 + fast)
    m, n, k, N = 130, 70, 150, 14
    A, B = randmat_np(rng, m, k), randmat_np(rng, k, n)
    C_tight, _, _ = run_gpu(A, B, N, fast=fast)
    lda, ldb, ldc = m + 7, k + 3, m + 5
    Ap = np.zeros((lda, k), order="F"); Ap[:m] = A
    Bp = np.zeros((ldb, n), order="F"); Bp[:k] = B
    Cp = np.full((ldc, n), 7.0, order="F")
    dA, dB, dC = to_dev(Ap), to_dev(Bp), to_dev(Cp)
    work = G.alloc_work(m, n, k, N)
    G.gemm(0, 0, m, n, k, 1.0, dA, lda, dB, ldb, 0.0, dC, ldc, N, fast, work)
    torch.cuda.synchronize()
    Cg = np.asfortranarray(dC.cpu().numpy().T)
    assert Cg[:m].tobytes() == C_tight.tobytes()
    assert np.all(Cg[m:] == 7.0)


@pytest.mark.parametrize("path", [0, 1, 3])
def test_residue_epilogue_exhaustive(path):
    """every input of the residue reductions of the product epilogue, all 20 moduli, against exact
    arithmetic: the biased form over x in [-2^30, 2^30] (k_pad <= 2^16) as integer Barrett (path 0) and
    as the f64 form the kernels use (path 3), and the reference's signed Barrett step
    (conv_32i_2_8u.hpp:7-56) over every int32 (path 1) -- 4.3e10, 4.3e10 and 8.6e10 checks"""
    import ctypes
    import gemmul8 as G
    G.lib.gemmul8_residue_selftest.restype = ctypes.c_ulonglong
    G.lib.gemmul8_residue_selftest.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert G.lib.gemmul8_residue_selftest(G._stream(), path) == 0
    if path == 0:  # negative control: a wrong expectation is counted for every (input, modulus) pair
        assert G.lib.gemmul8_residue_selftest(G._stream(), 2) == ((1 << 31) + 1) * 20


@pytest.mark.parametrize("N", [10, 11, 17, 18])
@pytest.mark.parametrize("fast", [True, False])
@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_encode_form_boundaries(N, fast, dt):
    """The encode switches residue forms by N (split.hip ModGroups): f64 pairs with one f32 step
    straight to bytes for N <= 17, triples with two steps above; f32 operands through the f64
    form for N <= 10 and mod_8i<float>'s four f32 steps above.  Wide dynamic range (phi = 3) and a
    row / column whose maximum dwarfs the rest put scaled values at the top of the magnitude range."""
    rng = np.random.default_rng(900 + N + 50 * fast + (dt == np.float32))
    m, n, k = 150, 130, 300
    A = randmat_np(rng, m, k, phi=3.0, dtype=dt)
    B = randmat_np(rng, k, n, phi=3.0, dtype=dt)
    A[5, :] *= dt(1e-6)
    A[5, 17] = dt(3.0e4)
    B[:, 9] *= dt(1e-5)
    B[200, 9] = dt(-7.0e3)
    check_full(A, B, N, fast=fast)


@pytest.mark.parametrize("N", [11, 14, 20])
@pytest.mark.parametrize("types", ["dsd", "sds", "zcz", "czc"])
def test_f32_four_step_encode_instantiation(N, types):
    """f32 operands above N = 10 in their own encode launch (operand types differ, so no pair kernel):
    the four-step-only instantiation (split.hip MODE 2), slices and output bit for bit against the oracle,
    with the same wide dynamic range as the form-boundary test"""
    ta, tb, tc = types
    rng = np.random.default_rng(1300 + N + 7 * ord(ta))
    m, n, k = 140, 110, 260
    A = randmat_np(rng, m, k, phi=3.0, dtype=_NPT[ta])
    B = randmat_np(rng, k, n, phi=3.0, dtype=_NPT[tb])
    if N > 19 and ta in "cz":
        N = 19  # complex fast mode with 20 moduli is a reference defect
    check_full(A, B, N, fast=True, out_dtype=_NPT[tc])


@pytest.mark.parametrize("fast", [True, False])
def test_offset_pointers(fast):
    """A, B and C one element past an allocation's start (8-byte aligned only) and the workspace 16
    bytes in (the reference assumes 16-byte alignment of `work`): same bits as aligned buffers"""
    torch = _torch()
    import gemmul8 as G
    rng = np.random.default_rng(91 + fast)
    m, n, k, N = 130, 70, 150, 14
    A, B = randmat_np(rng, m, k), randmat_np(rng, k, n)
    C_ref, _, _ = run_gpu(A, B, N, fast=fast)

    def dev_offset(X):
        flat = torch.zeros(X.size + 1, dtype=torch.float64, device="cuda")
        flat[1:] = torch.from_numpy(np.asfortranarray(X).reshape(-1, order="F")).cuda()
        return flat[1:]

    dA, dB = dev_offset(A), dev_offset(B)
    dC = dev_offset(np.zeros((m, n)))
    wbuf = torch.empty(G.workSize(m, n, k, N) + 16, dtype=torch.uint8, device="cuda")
    G.gemm(0, 0, m, n, k, 1.0, dA, m, dB, k, 0.0, dC, m, N, fast, wbuf[16:])
    torch.cuda.synchronize()
    Cg = dC.cpu().numpy().reshape((m, n), order="F")
    assert np.asfortranarray(Cg).tobytes() == np.asfortranarray(C_ref).tobytes()


@pytest.mark.parametrize("fast", [True, False])
def test_integer_inputs_at_scale(fast):
    """Size-independent property at a size the oracle cannot check quickly: for integer inputs the
    exact product is known (float64 matmul of integers below 2^53 is exact), and the emulation
    must stay within the Ozaki-II bound |C - AB| <= 2^-44 (|A| |B|) elementwise (its error is the
    CRT's double-double rounding only: measured 6e-12 relative on the oracle-checked small case,
    tools/probes/intcheck.py).  16384 x 12288 x 1536 real, 4096 x 3072 x 1024 complex."""
    torch = _torch()
    import gemmul8 as G
    g = torch.Generator(device="cuda").manual_seed(1234 + fast)

    def check(C, exact, bound):
        err = (C - exact).abs()
        assert bool((err <= bound * 2.0 ** -44).all()), float((err / bound).max())

    m, n, k = 16384, 12288, 1536
    A = torch.randint(-1000, 1001, (k, m), generator=g, device="cuda").to(torch.float64)  # column-major m x k
    B = torch.randint(-1000, 1001, (n, k), generator=g, device="cuda").to(torch.float64)  # column-major k x n
    C = torch.empty((n, m), dtype=torch.float64, device="cuda")
    W = G.alloc_work(m, n, k, 14)
    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, fast, W)
    check(C, B @ A, B.abs() @ A.abs())  # (n x k)(k x m): the column-major A B
    del W, C
    mc, nc, kc = 4096, 3072, 1024
    Ac = torch.complex(torch.randint(-500, 501, (kc, mc), generator=g, device="cuda").double(),
                       torch.randint(-500, 501, (kc, mc), generator=g, device="cuda").double())
    Bc = torch.complex(torch.randint(-500, 501, (nc, kc), generator=g, device="cuda").double(),
                       torch.randint(-500, 501, (nc, kc), generator=g, device="cuda").double())
    Cc = torch.empty((nc, mc), dtype=torch.complex128, device="cuda")
    Wc = G.alloc_work(mc, nc, kc, 12, G.COMPLEX_BIG_MATRIX_ENCODE)
    G.gemm(0, 0, mc, nc, kc, 1.0, Ac, mc, Bc, kc, 0.0, Cc, mc, 12, fast, Wc, G.COMPLEX_BIG_MATRIX_ENCODE)
    check(Cc, Bc @ Ac, 2.0 * (Bc.abs() @ Ac.abs()))


@pytest.mark.parametrize("dt", [np.complex128, np.complex64])
@pytest.mark.parametrize("alpha,beta", [(1.0, 1.0), (2.0, 0.5), (1.0, -3.0), (1.5 - 0.5j, 0.25 + 0.75j)])
def test_complex_nonfinite_imag_c(dt, alpha, beta):
    """Complex C whose imaginary parts hold Inf: bits equal to the oracle, which restates the
    reference's epilogue kernels (tests/test_oracle_epilogue.py).  alpha = beta = 1 is the reference's
    component-wise CAdd (inverse_scaling.hpp:370-392), so Re(C) stays finite there; the hipCfma forms
    of the other variants carry the Inf into Re(C) (0 * Inf = NaN for a real beta), as the reference does."""
    rng = np.random.default_rng(404 + (dt == np.complex64))
    m, n, k = 40, 30, 50
    A, B = randmat_np(rng, m, k, dtype=dt), randmat_np(rng, k, n, dtype=dt)
    C0 = randmat_np(rng, m, n, dtype=dt)
    C0.imag[3, 4] = np.inf
    C0.imag[7, 1] = -np.inf
    C0.imag[0, 0] = np.inf
    C, Co = check_full(A, B, 9, alpha=alpha, beta=beta, C0=C0)
    if (alpha, beta) == (1.0, 1.0):
        assert np.isfinite(C.real).all()
        assert np.isinf(C.imag[3, 4]) and np.isinf(C.imag[7, 1])
    else:
        assert not np.isfinite(C.real[3, 4]) and not np.isfinite(C.real[7, 1])


def test_stale_hip_error_is_not_reported():
    """An error left pending on the thread by an earlier, unrelated HIP call (here a failed
    hipSetDevice) is neither reported as the call's own nor consumed: the call succeeds, writes the
    correct bits with beta != 0, and the application still finds its own error pending afterwards."""
    import ctypes
    torch = _torch()
    hip = ctypes.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_LAZY)
    rng = np.random.default_rng(77)
    m, n, k = 96, 80, 130
    A, B, C0 = randmat_np(rng, m, k), randmat_np(rng, k, n), randmat_np(rng, m, n)
    from oracle import oracle as O
    Co = O.gemm(A, B, 14, True, np.float64, 1.0, 0.5, C0)
    import gemmul8 as G
    dA, dB, dC = to_dev(A), to_dev(B), to_dev(C0)
    work = G.alloc_work(m, n, k, 14)
    torch.cuda.synchronize()
    assert hip.hipSetDevice(ctypes.c_int(12345)) != 0
    assert hip.hipPeekAtLastError() != 0  # the stale error is pending
    G.gemm(0, 0, m, n, k, 1.0, dA, m, dB, k, 0.5, dC, m, 14, True, work)  # raises on a nonzero return
    assert hip.hipPeekAtLastError() != 0  # still the application's to read
    assert hip.hipGetLastError() != 0
    torch.cuda.synchronize()
    assert bits_equal(np.asfortranarray(dC.cpu().numpy().T), Co)


def test_persistent_products_forced():
    """GEMMUL8_PERSISTENT=1 (child process): the persistent residue kernel (per-XCD tile queues,
    k-step pipeline across tiles, residue stores in flight under the next tile) at small shapes,
    also with the grid capped to 16 blocks (GEMMUL8_PERSISTENT_GRID) so every block walks many
    tiles and the queues of four XCDs stay empty; slices, residues and C against the oracle for
    real f64 / f32, accurate mode, the signed residue path (k_pad > 2^16), Karatsuba complex
    sub-products, and low-memory mode (several product launches on one workspace); the workspace
    starts as 0xA5 bytes, so the queue heads are garbage until the launch zeroes them"""
    import subprocess
    code = ("import sys, numpy as np; sys.path[:0] = sys.argv[1:4]\n"
            "from test_gpu_parity import check_full\nfrom util import randmat_np\n"
            "import gemmul8 as G, torch\n"
            "rng = np.random.default_rng(23)\n"
            "check_full(randmat_np(rng, 300, 513), randmat_np(rng, 513, 260), 14)\n"
            "check_full(randmat_np(rng, 300, 300), randmat_np(rng, 300, 260), 14)\n"  # 5 k-steps per tile
            "check_full(randmat_np(rng, 300, 330), randmat_np(rng, 330, 260), 14)\n"  # 6 k-steps per tile
            "check_full(randmat_np(rng, 700, 333), randmat_np(rng, 333, 530), 9, fast=False)\n"
            "check_full(randmat_np(rng, 520, 400, dtype=np.float32), randmat_np(rng, 400, 270, dtype=np.float32), 7)\n"
            "check_full(randmat_np(rng, 20, 70000), randmat_np(rng, 70000, 24), 14)\n"
            "check_full(randmat_np(rng, 300, 333, dtype=np.complex128), randmat_np(rng, 333, 290, dtype=np.complex128), 12, ctype=3)\n"
            "m, n, k, N = 600, 520, 700, 14\n"
            "A = torch.randn((k, m), dtype=torch.float64, device='cuda'); B = torch.randn((n, k), dtype=torch.float64, device='cuda')\n"
            "Cs = []\n"
            "for S in (None, 3):\n"
            "    W = G.alloc_work(m, n, k, N, 0, slice_planes=S); W.fill_(0xA5); C = torch.empty((n, m), dtype=torch.float64, device='cuda')\n"
            "    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, True, W, 0, slice_planes=S); Cs.append(C.cpu())\n"
            "assert torch.equal(Cs[0], Cs[1])\n"
            "print('OK')")
    tdir = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(tdir)
    # the per-group-epilogue kernel (default) with and without a capped grid, and the block-epilogue kernel
    for cap, pg in (("", "1"), ("16", "1"), ("16", "0")):
        env = dict(os.environ, GEMMUL8_PERSISTENT="1", GEMMUL8_PERSISTENT_GRID=cap, GEMMUL8_CPLX_PRODUCTS="karatsuba",
                   GEMMUL8_PG_EPILOGUE=pg)
        r = subprocess.run([sys.executable, "-c", code, tdir, root, os.path.join(root, "mixed-gemmul8_amd")], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "OK" in r.stdout, (cap, pg, r.stderr[-3000:])


def test_persistent_default_matches_one_tile():
    """Production shapes where the default rule picks the persistent residue kernel (>= 3 tiles per
    CU): C bit-identical to the one-tile kernel (GEMMUL8_PERSISTENT=0, child process) at k-steps per
    tile around the kernel's minimum (5: one-tile kernel; 6, 7, 128: persistent), and at 2048^3
    (3.5 tiles per CU: blocks with different tile counts).  With 5 k-steps the persistent kernel's
    DMA cursor used to jump to the next tile before it was decoded."""
    import subprocess
    import tempfile
    tdir = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(tdir)
    code = ("import sys, numpy as np, torch; sys.path[:0] = sys.argv[1:3]\n"
            "import gemmul8 as G\n"
            "out = sys.argv[3]; res = {}\n"
            "for m, k in ((4096, 300), (4096, 330), (4096, 400), (4096, 8192), (2048, 2048)):\n"
            "    n = m\n"
            "    g = torch.Generator(device='cuda'); g.manual_seed(k)\n"
            "    A = torch.randn((k, m), dtype=torch.float64, device='cuda', generator=g)\n"
            "    B = torch.randn((n, k), dtype=torch.float64, device='cuda', generator=g)\n"
            "    C = torch.empty((n, m), dtype=torch.float64, device='cuda')\n"
            "    W = G.alloc_work(m, n, k, 14)\n"
            "    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, True, W)\n"
            "    res[f'{m}_{k}'] = C.cpu().numpy()\n"
            "np.savez(out, **res)\n")
    with tempfile.TemporaryDirectory() as d:
        outs = []
        for mode in ("0", ""):
            out = os.path.join(d, f"c{mode or 'default'}.npz")
            env = dict(os.environ, GEMMUL8_PERSISTENT=mode) if mode else {
                kk: v for kk, v in os.environ.items() if kk != "GEMMUL8_PERSISTENT"}
            r = subprocess.run([sys.executable, "-c", code, os.path.join(root, "mixed-gemmul8_amd"), tdir, out],
                               env=env, capture_output=True, text=True, timeout=300)
            assert r.returncode == 0, r.stderr[-3000:]
            outs.append(np.load(out))
        for k in outs[0].files:
            assert np.array_equal(outs[0][k].view(np.uint64), outs[1][k].view(np.uint64)), k


def test_small_tiles_match_one_tile():
    """The 128 x 128-tile product kernel (gemm_i8_small_kernel; by default the accurate-mode bound product below
    one 256 x 256 tile per CU): C bit-identical to the 256-tile one-tile kernel (GEMMUL8_SMALL_TILES=0
    GEMMUL8_PERSISTENT=0) and the rule's default, child processes, at 1024^3, odd shapes with partial 128-tiles, k
    from 1 k-step to 33, accurate mode (the bound product runs the small kernel too), f32, Karatsuba complex
    sub-products, and with the kernel forced wherever it applies (GEMMUL8_SMALL_TILES=1: 2048^3, 3.5 tiles of
    256 x 256 per CU); the oracle checks the forced small kernel's slices, residues and C at small shapes"""
    import subprocess
    import tempfile
    tdir = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(tdir)
    code = ("import sys, numpy as np, torch; sys.path[:0] = sys.argv[1:3]\n"
            "import gemmul8 as G\n"
            "out = sys.argv[3]; res = {}\n"
            "cases = ((1024, 1024, 1024, 14, True, 'd', 0), (300, 200, 64, 14, True, 'd', 0),\n"
            "         (900, 130, 2100, 14, True, 'd', 0), (1024, 1024, 1024, 14, False, 'd', 0),\n"
            "         (700, 540, 333, 9, False, 'd', 0), (520, 270, 400, 7, True, 'f', 0),\n"
            "         (1024, 300, 3072, 12, True, 'z', 3), (2048, 2048, 2048, 14, True, 'd', 0),\n"
            "         (1152, 1152, 1152, 14, True, 'd', 0), (1152, 1152, 1152, 14, False, 'd', 0))\n"
            "for m, n, k, N, fast, t, ct in cases:\n"
            "    dt = {'d': torch.float64, 'f': torch.float32, 'z': torch.complex128}[t]\n"
            "    g = torch.Generator(device='cuda'); g.manual_seed(m + n + k)\n"
            "    A = torch.randn((k, m), dtype=dt, device='cuda', generator=g)\n"
            "    B = torch.randn((n, k), dtype=dt, device='cuda', generator=g)\n"
            "    C = torch.empty((n, m), dtype=dt, device='cuda')\n"
            "    W = G.alloc_work(m, n, k, N, ct)\n"
            "    G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, W, ct)\n"
            "    res[f'{m}_{n}_{k}_{N}_{fast}_{t}'] = C.cpu().numpy()\n"
            "    res[f'{m}_{n}_{k}_{N}_{fast}_{t}_kernel'] = np.array([G.last_products_kernel()])\n"
            "np.savez(out, **res)\n")
    modes = {"onetile": {"GEMMUL8_SMALL_TILES": "0", "GEMMUL8_PERSISTENT": "0"}, "default": {},
             "forced": {"GEMMUL8_SMALL_TILES": "1"}, "tail": {"GEMMUL8_TAIL_SMALL": "1"}}
    with tempfile.TemporaryDirectory() as d:
        outs = {}
        for name, extra in modes.items():
            out = os.path.join(d, f"{name}.npz")
            env = {kk: v for kk, v in os.environ.items()
                   if kk not in ("GEMMUL8_SMALL_TILES", "GEMMUL8_PERSISTENT", "GEMMUL8_TAIL_SMALL")}
            env.update(extra)
            r = subprocess.run([sys.executable, "-c", code, os.path.join(root, "mixed-gemmul8_amd"), tdir, out],
                               env=env, capture_output=True, text=True, timeout=300)
            assert r.returncode == 0, (name, r.stderr[-3000:])
            outs[name] = np.load(out)
        for key in outs["onetile"].files:
            if key.endswith("_kernel"):
                continue
            for name in ("default", "forced", "tail"):
                assert np.array_equal(outs["onetile"][key].view(np.uint8), outs[name][key].view(np.uint8)), (name, key)
        assert str(outs["forced"]["2048_2048_2048_14_True_d_kernel"][0]) == "gemm_i8_small_kernel"
        assert str(outs["forced"]["1024_1024_1024_14_True_d_kernel"][0]) == "gemm_i8_small_kernel"
        # (1024^3: 224 tiles on 256 CUs, at most 1.5 per CU: the persistent per-group kernel since round 6)
        assert str(outs["default"]["1024_1024_1024_14_True_d_kernel"][0]) == "gemm_i8_persistent_pg_kernel"
        assert str(outs["default"]["2048_2048_2048_14_True_d_kernel"][0]) == "gemm_i8_persistent_pg_kernel"
        # tail planes: 2048^3 (3.5 tiles per CU) 12 planes on the persistent kernel (3 rounds), the last 2 as
        # 128 x 128 tiles; 1152^3 (350 tiles on 256 CUs) 10 planes on the one-tile kernel (250 tiles: uneven XCD
        # shares of 25 tiles per plane would take the persistent kernel two rounds) and 4 as 128 x 128 tiles
        assert str(outs["tail"]["2048_2048_2048_14_True_d_kernel"][0]) == \
            "gemm_i8_persistent_pg_kernel+gemm_i8_small_kernel"
        assert str(outs["tail"]["1152_1152_1152_14_True_d_kernel"][0]) == "gemm_i8_kernel+gemm_i8_small_kernel"
        assert str(outs["onetile"]["1024_1024_1024_14_True_d_kernel"][0]) == "gemm_i8_kernel"
    code = ("import sys, numpy as np; sys.path[:0] = sys.argv[1:4]\n"
            "from test_gpu_parity import check_full\nfrom util import randmat_np\n"
            "rng = np.random.default_rng(29)\n"
            "check_full(randmat_np(rng, 300, 513), randmat_np(rng, 513, 260), 14)\n"
            "check_full(randmat_np(rng, 130, 64), randmat_np(rng, 64, 129), 14)\n"
            "check_full(randmat_np(rng, 700, 333), randmat_np(rng, 333, 530), 9, fast=False)\n"
            "check_full(randmat_np(rng, 520, 400, dtype=np.float32), randmat_np(rng, 400, 270, dtype=np.float32), 7)\n"
            "check_full(randmat_np(rng, 300, 333, dtype=np.complex128), randmat_np(rng, 333, 290, dtype=np.complex128), 12, ctype=3)\n"
            "print('OK')")
    for extra in ({"GEMMUL8_SMALL_TILES": "1", "GEMMUL8_CPLX_PRODUCTS": "karatsuba"},
                  {"GEMMUL8_SMALL_TILES": "0", "GEMMUL8_PERSISTENT": "0"}):
        env = dict(os.environ, **extra)
        r = subprocess.run([sys.executable, "-c", code, tdir, root, os.path.join(root, "mixed-gemmul8_amd")], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "OK" in r.stdout, (extra, r.stderr[-3000:])


def test_persistent_planes_beyond_4gib():
    """A launch whose 14 A slice planes span more than 4 GiB (m = 20480, k = 15360: 315 MB per plane):
    the persistent kernel addresses each modulus's plane with its own buffer descriptor and switches
    descriptors with its DMA cursor; C bit-identical to the one-tile kernel (GEMMUL8_PERSISTENT=0)."""
    import subprocess
    import tempfile
    tdir = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(tdir)
    code = ("import sys, numpy as np, torch; sys.path[:0] = sys.argv[1:3]\n"
            "import gemmul8 as G\n"
            "m, n, k, N = 20480, 256, 15360, 14\n"
            "assert N * G.layout(m, n, k, N)['planeA'] > (1 << 32)\n"
            "g = torch.Generator(device='cuda'); g.manual_seed(5)\n"
            "A = torch.randn((k, m), dtype=torch.float64, device='cuda', generator=g)\n"
            "B = torch.randn((n, k), dtype=torch.float64, device='cuda', generator=g)\n"
            "C = torch.empty((n, m), dtype=torch.float64, device='cuda')\n"
            "W = G.alloc_work(m, n, k, N)\n"
            "G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, True, W)\n"
            "np.save(sys.argv[3], C.cpu().numpy())\n")
    with tempfile.TemporaryDirectory() as d:
        outs = []
        for mode in ("0", ""):
            out = os.path.join(d, f"c{mode or 'default'}.npy")
            env = dict(os.environ, GEMMUL8_PERSISTENT=mode) if mode else {
                kk: v for kk, v in os.environ.items() if kk != "GEMMUL8_PERSISTENT"}
            r = subprocess.run([sys.executable, "-c", code, os.path.join(root, "mixed-gemmul8_amd"), tdir, out],
                               env=env, capture_output=True, text=True, timeout=300)
            assert r.returncode == 0, r.stderr[-3000:]
            outs.append(np.load(out))
        assert np.array_equal(outs[0].view(np.uint64), outs[1].view(np.uint64))


@pytest.mark.parametrize("fast", [True, False])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_nonfinite_inputs(fast, dtype):
    """NaN / +-Inf in A and B: shifts, slices, residues and C equal the oracle's bit for bit (the
    live comparison with the reference's build is tests/test_ref_parity.py::test_nonfinite_inputs_same_bits)."""
    rng = np.random.default_rng(31)
    A, B = randmat_np(rng, 70, 90).astype(dtype), randmat_np(rng, 90, 50).astype(dtype)
    A[4, 10] = np.nan
    A[9, 3] = np.inf
    B[7, 8] = -np.inf
    B[20, 30] = np.nan
    check_full(A, B, 12 if dtype == np.float64 else 7, fast=fast)


def _magnitude_edge_rows(X, dtype):
    """Rows of X (n_vec x k, k >= 256) that exercise the accurate mode's one-read magnitudes (split.hip
    mag_tile_kernel / mag_fixup_kernel): tile amax below the vector amax by d = 1..7 and beyond, elements at and
    across the subnormal boundary of the final scale, Inf / NaN in one tile, all-NaN, all-zero and -0.0 rows,
    a 2^2000 (f64) dynamic range, magnitudes of exactly 64."""
    dbl = dtype == np.float64
    emin = -1022 if dbl else -126
    X[1, :64] *= 1.0
    X[1, 64:] *= 2.0 ** -17           # tiles 1.. : d = 17 (every nonzero byte -> 1)
    X[2, 64:128] *= 0.3               # d = 1 or 2
    X[2, 128:192] *= 2.0 ** -5        # d ~ 5
    X[3, :] = 0.75
    X[3, 100] = 2.0 ** (emin + 22)    # far from the boundary: exact path
    X[4, :] = 0.75                    # amax 0.75: final scale 2^6
    X[4, 150] = 2.0 ** (emin - 6)     # a subnormal input scaled exactly onto the least normal exponent: exact path
    X[5, :] = 0.75
    X[5, 70] = 2.0 ** (emin - 7)      # one below (subnormal under the final scale): recomputed from the operand
    X[5, 71] = 2.0 ** (emin - 20)
    X[6, 200] = np.inf
    X[7, 90] = np.nan
    X[8, :] = np.nan
    X[9, :] = 0.0
    X[10, :] = -0.0
    X[10, 5] = 1.5
    X[10, 130] = -0.0
    if dbl:
        X[11, :64] *= 1e300
        X[11, 64:128] *= 1e-300
    else:
        X[11, :64] *= 1e30
        X[11, 64:128] *= 1e-30
    X[12, :] = 63.5                  # amax 63.5 -> sft0 = 0: bytes of 64
    X[12, 64:] = 0.99                # tile amax below: d = 5
    return X


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("opA,opB", [(0, 0), (1, 1)])
def test_accurate_magnitudes_one_read_edges(dtype, opA, opB):
    """Accurate mode's sft0 and magnitudes from one read of each operand (pass 1 scales by the tile amax, pass 2
    rescales the bytes or recomputes the tile): shifts, slices, residues and C against the oracle at the edges of
    that scheme, for strided (op N A, op T B) and contiguous (op T A, op N B) vectors."""
    rng = np.random.default_rng(77)
    m, n, k = 40, 36, 300
    A = _magnitude_edge_rows(randmat_np(rng, m, k).astype(dtype), dtype)
    Bt = _magnitude_edge_rows(randmat_np(rng, n, k).astype(dtype), dtype)  # rows of B^T = columns of B
    A = np.asfortranarray(A.T) if opA else np.asfortranarray(A)
    B = np.asfortranarray(Bt) if opB else np.asfortranarray(Bt.T)
    check_full(A, B, 10 if dtype == np.float64 else 7, fast=False, opA=opA, opB=opB)
