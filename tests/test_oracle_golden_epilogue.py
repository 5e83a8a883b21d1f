"""CPU: the oracle's BLAS epilogue against the REFERENCE's own outputs for general and complex alpha / beta
(tests/golden/ref_golden_epilogue.npz, made by tests/golden/make_golden_epilogue.py with the reference's
build on an MI355X): real and complex, one- and two-level moduli, the _a1 / _ab / CAdd kernels
(inverse_scaling.hpp:268-948).  C must match byte for byte."""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_golden_epilogue.npz")
_D = np.load(GOLD)  # no pickles (allow_pickle defaults to False)
NAMES = sorted({k.split("/")[0] for k in _D.files})


@pytest.mark.parametrize("name", NAMES)
def test_epilogue_matches_reference(name):
    g = {k.split("/")[1]: _D[k] for k in _D.files if k.startswith(name + "/")}
    assert int(g["rc"][0]) == 0
    A, B, C0, C = g["A"], g["B"], g["C0"], g["C"]
    al, be = g["alpha"][0], g["beta"][0]
    C_or = O.gemm(A, B, int(g["N"][0]), True, C.dtype, al, be, C0)
    assert C_or.tobytes() == np.asfortranarray(C).tobytes(), \
        f"{int(np.sum(C_or != C))} elements differ from the reference"


def test_fixture_covers_the_variants():
    assert len(NAMES) >= 20
    cplx = [n for n in NAMES if n[0] in "zc"]
    assert any(n.startswith("z_N14") for n in cplx) and any(n.startswith("z_N6") for n in cplx)
