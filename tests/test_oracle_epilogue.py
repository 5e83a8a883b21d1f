"""CPU: the oracle's complex BLAS epilogue (oracle/oz2_oracle.c cepi_d / cepi_f), which restates the
reference's kernels operation for operation (GEMMul8/src/inverse_scaling.hpp:268-948) with hip_complex.h's
hipCmul / hipCfma as clang contracts them in the reference's build:
    hipCmul(p, q)    = (fma(p.x, q.x, -(p.y*q.y)), fma(p.y, q.x, p.x*q.y))   (two-level f64: fma(p.x, q.y, p.y*q.x))
    hipCfma(p, q, r) = (fma(-p.y, q.y, fma(p.x, q.x, r.x)), fma(p.x, q.y, fma(q.x, p.y, r.y)))
    alpha = 1, beta = 0: v;  alpha = beta = 1: C + v (CAdd);  beta = 1: hipCfma(alpha, v, C);
    otherwise hipCfma(beta, C, hipCmul(alpha, v)); beta = 0 never reads C (BLAS).
The forms were pinned on the reference's own full-precision outputs (tools/probes/epi_dump2.py, searched
over every contraction) and by tests/golden/ref_golden_epilogue.npz (tests/test_oracle_golden_epilogue.py); the live comparison is tests/test_ref_parity.py."""
from fractions import Fraction as Fr

import numpy as np
import pytest

from oracle import oracle as O
from util import randmat_np


def _fma(a, b, c):  # correctly rounded f64 fma (exact rational arithmetic)
    if not all(np.isfinite([a, b, c])):
        return a * b + c
    return float(Fr(a) * Fr(b) + Fr(c))


def _cmul(pr, pi, qr, qi, two_level):
    if two_level:  # numM = 2 complex-double kernels
        return _fma(pr, qr, -(pi * qi)), _fma(pr, qi, pi * qr)
    return _fma(pr, qr, -(pi * qi)), _fma(pi, qr, pr * qi)


def _cfma(pr, pi, qr, qi, rr, ri):
    re, im = _fma(pr, qr, rr), _fma(qr, pi, ri)
    return _fma(-pi, qi, re), _fma(pr, qi, im)


def _expected(v, c, al, be, two_level):
    ar, ai, br, bi = al.real, al.imag, be.real, be.imag
    a1 = ar == 1 and ai == 0
    x = (v.real, v.imag) if a1 else _cmul(ar, ai, v.real, v.imag, two_level)
    if br == 0 and bi == 0:
        return x
    if br == 1 and bi == 0:
        return (c.real + v.real, c.imag + v.imag) if a1 else _cfma(ar, ai, v.real, v.imag, c.real, c.imag)
    return _cfma(br, bi, c.real, c.imag, x[0], x[1])


@pytest.mark.parametrize("N", [6, 14])  # one- and two-level moduli
@pytest.mark.parametrize("al,be", [(1.5 - 0.5j, 0.0), (1.5 - 0.5j, 0.25 + 0.75j), (1.0 + 1.0j, 1.0), (2.5, 1.0),
                                   (2.5, 0.5), (1.0, 1.0), (1.0, -3.0 + 0.5j), (0.3 + 1.7j, -1.25 + 0.5j)])
def test_epilogue_forms_bit_exact(al, be, N):
    rng = np.random.default_rng(5)
    m, n, k = 12, 9, 20
    A, B = randmat_np(rng, m, k, dtype=np.complex128), randmat_np(rng, k, n, dtype=np.complex128)
    C0 = randmat_np(rng, m, n, dtype=np.complex128)
    V = O.gemm(A, B, N, True, np.complex128)  # alpha = 1, beta = 0: the unscaled product
    C = O.gemm(A, B, N, True, np.complex128, al, be, C0)
    al, be = complex(al), complex(be)
    for i in range(m):
        for j in range(n):
            er, ei = _expected(V[i, j], C0[i, j], al, be, N == 14)
            assert (C[i, j].real, C[i, j].imag) == (er, ei), (i, j)


@pytest.mark.parametrize("dt", [np.complex128, np.complex64])
def test_alpha_beta_one_keeps_components_apart(dt):
    """alpha = beta = 1 is the reference's component-wise CAdd: a non-finite Im(C) stays out of Re(C)."""
    rng = np.random.default_rng(6)
    A, B = randmat_np(rng, 10, 14, dtype=dt), randmat_np(rng, 14, 8, dtype=dt)
    C0 = randmat_np(rng, 10, 8, dtype=dt)
    C0.imag[2, 3] = np.inf
    C0.imag[5, 0] = np.nan
    C = O.gemm(A, B, 12, True, dt, 1.0, 1.0, C0)
    AB = O.gemm(A, B, 12, True, dt)
    assert C.real.tobytes() == (C0.real + AB.real).tobytes()
    assert np.isfinite(C.real).all()


@pytest.mark.parametrize("dt", [np.complex128, np.complex64])
@pytest.mark.parametrize("alpha,beta", [(2.0, 0.5), (2.5, 1.0)])
def test_nonfinite_imag_c_as_the_reference(dt, alpha, beta):
    """Other (alpha, beta) go through hipCfma, whose -(p.y*q.y) / (q.x*p.y) terms turn a non-finite
    Im(C) into NaN in Re(C) exactly as the reference's _ab / _a1 kernels do; elsewhere C is finite."""
    rng = np.random.default_rng(7)
    A, B = randmat_np(rng, 10, 14, dtype=dt), randmat_np(rng, 14, 8, dtype=dt)
    C0 = randmat_np(rng, 10, 8, dtype=dt)
    C0.imag[2, 3] = np.inf
    C = O.gemm(A, B, 9, True, dt, alpha, beta, C0)
    bad = np.zeros(C.shape, bool)
    bad[2, 3] = True
    assert np.isfinite(C[~bad]).all()
    AB = O.gemm(A, B, 9, True, dt)
    tol = 1e-5 if dt == np.complex64 else 1e-13
    with np.errstate(invalid="ignore"):  # beta * C0 at the Inf element (masked out)
        expect = alpha * AB + beta * C0
    assert np.allclose(C[~bad], expect[~bad], rtol=tol)
