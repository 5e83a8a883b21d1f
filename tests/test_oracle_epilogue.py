"""CPU: the oracle's complex BLAS epilogue (oracle/oz2_oracle.c oz2o_crt).  With real alpha and beta
each component takes the real-scalar form: alpha = beta = 1 is the reference's component-wise CAdd
(GEMMul8/src/inverse_scaling.hpp:370-392), and a non-finite Im(C) cannot turn Re(C) into NaN through a
0 * Inf term of the full complex product.  Complex alpha keeps the complex form."""
import numpy as np
import pytest

from oracle import oracle as O
from util import randmat_np


@pytest.mark.parametrize("dt", [np.complex128, np.complex64])
@pytest.mark.parametrize("alpha,beta", [(1.0, 1.0), (2.0, 0.5), (-1.0, 3.0)])
def test_real_scalars_keep_components_apart(dt, alpha, beta):
    rng = np.random.default_rng(5)
    m, n, k = 12, 9, 20
    A, B = randmat_np(rng, m, k, dtype=dt), randmat_np(rng, k, n, dtype=dt)
    C0 = randmat_np(rng, m, n, dtype=dt)
    C0.imag[2, 3] = np.inf
    C0.imag[5, 0] = np.nan
    C = O.gemm(A, B, 9, True, dt, alpha, beta, C0)
    assert np.isfinite(C.real).all()
    AB = O.gemm(A, B, 9, True, dt)
    finite = np.isfinite(C0.imag)
    rd = np.float64 if dt == np.complex128 else np.float32
    # each component: fma(beta, c, alpha * v), exact to one rounding of the real form
    exp_re = (rd(beta) * C0.real.astype(rd) + rd(alpha) * AB.real).astype(rd)
    assert np.allclose(C.real, exp_re, rtol=1e-6 if rd == np.float32 else 1e-14, atol=0)
    assert np.allclose(C.imag[finite], (rd(beta) * C0.imag + rd(alpha) * AB.imag)[finite],
                       rtol=1e-6 if rd == np.float32 else 1e-14)


def test_alpha_beta_one_is_componentwise_add():
    rng = np.random.default_rng(6)
    A, B = randmat_np(rng, 10, 14, dtype=np.complex128), randmat_np(rng, 14, 8, dtype=np.complex128)
    C0 = randmat_np(rng, 10, 8, dtype=np.complex128)
    C = O.gemm(A, B, 12, True, np.complex128, 1.0, 1.0, C0)
    AB = O.gemm(A, B, 12, True, np.complex128)
    assert C.real.tobytes() == (C0.real + AB.real).tobytes()
    assert C.imag.tobytes() == (C0.imag + AB.imag).tobytes()


def test_complex_alpha_keeps_complex_form():
    rng = np.random.default_rng(7)
    A, B = randmat_np(rng, 10, 14, dtype=np.complex128), randmat_np(rng, 14, 8, dtype=np.complex128)
    C0 = randmat_np(rng, 10, 8, dtype=np.complex128)
    al, be = 0.5 - 1.25j, 2.0 + 0.5j
    C = O.gemm(A, B, 12, True, np.complex128, al, be, C0)
    AB = O.gemm(A, B, 12, True, np.complex128)
    assert np.allclose(C, al * AB + be * C0, rtol=1e-13)
