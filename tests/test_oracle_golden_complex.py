"""The CPU oracle against golden vectors of the REFERENCE's complex compute types
(tests/golden/ref_golden_complex.npz, written by tests/golden/make_golden_complex.py from the
reference's own HIP build on MI355X).

Expectation: identical shifts and bit-identical C, except for documented reference defects
(DESIGN.md section 10):
  * COMPLEX_CLASSIC_MULT / COMPLEX_KARATSUBA_MULT with a complex-double output and
    num_moduli >= 8: the reference's CRT for these types only implements the single-double
    path (inverse_scaling.hpp:1031-1062 commented out) and never writes C (shifts compared);
  * COMPLEX_BIG_MATRIX_ENCODE, fast mode, num_moduli = 20: O(1) errors in the reference;
  * accurate mode, big matrix, op(A) = T: the row bound is read from column r of the bound
    product (scalingB_kernel_bigmatrix_minusBL launched with (n, k, m), scaling.hpp:3233-3235);
    op(B) = T: the column bound from row c (scalingA_kernel_bigmatrix_minusTR with (m, n, k),
    :3236-3238); op(A) = C with m != n: the bottom big-matrix rows are written at row offset n
    (extract_B8i_kernel_bigmatrix(k, n, ...), :3207-3209);
  * accurate mode, classic / Karatsuba, op(A) = C: A's imaginary magnitudes are written into
    B8i_imag (scaling.hpp:3320), so both bounds are off.
In those shift-defect cases the oracle's shifts follow the reference's evident intent (correct
row / column bounds, the reference's sign rule for op C) and its product must be accurate.
The classic and Karatsuba types are checked against the oracle's big-matrix computation: all
three compute types produce the same residues.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_golden_complex.npz")
NPT = {"z": np.complex128, "c": np.complex64}
OPS = {0: lambda X: X, 1: lambda X: X.T, 2: lambda X: X.conj().T}


def _cases():
    if not os.path.exists(GOLD):
        return []
    g = np.load(GOLD)
    return sorted({k.split("/")[0] for k in g.files})


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def reference_defect(name, tc, N, fast, ctype, opA, opB):
    if ctype in (2, 3) and tc == "z" and N >= 8:
        return "classic/Karatsuba double-double CRT missing: C never written"
    if ctype == 1 and fast and N == 20:
        return "big-matrix fast mode, 20 moduli: O(1) errors"
    return None


def shift_defect(ctype, fast, opA, opB, m, n):
    """which of the reference's shift arrays is wrong (accurate complex op T / C), or None"""
    if fast:
        return None
    if ctype == 1:
        bad = set()
        if opA == 1 or (opA == 2 and m != n):
            bad.add("A")
        if opB == 1:
            bad.add("B")
        return bad or None
    if opA == 2:
        return {"A", "B"}
    return None


@pytest.mark.parametrize("name", _cases())
def test_oracle_matches_reference_complex(gold, name):
    A, B, C = gold[name + "/A"], gold[name + "/B"], gold[name + "/C"]
    opA, opB, m, n, k, N, fast, ctype = (int(x) for x in gold[name + "/meta"])
    tc = str(gold[name + "/types"][0])[2]
    Co, sA, sB = O.gemm(A, B, N, bool(fast), NPT[tc], opA=opA, opB=opB, return_sft=True, ctype=ctype)
    exact = OPS[opA](A.astype(np.complex128)) @ OPS[opB](B.astype(np.complex128))
    err = np.max(np.abs(Co - exact) / np.abs(exact))
    assert err < (1e-5 if tc == "c" else 1e-7), err
    bad = shift_defect(ctype, fast, opA, opB, m, n)
    if bad:
        # the defective side's shifts must differ from ours (the defect is live in this case),
        # the other side's must agree
        for side, mine in (("A", sA), ("B", sB)):
            same = np.array_equal(mine, gold[name + "/sft" + side])
            assert same != (side in bad), f"sft{side}: expected {'a difference' if side in bad else 'agreement'}"
        return
    assert np.array_equal(sA, gold[name + "/sftA"]), "sftA differs from the reference"
    assert np.array_equal(sB, gold[name + "/sftB"]), "sftB differs from the reference"
    why = reference_defect(name, tc, N, fast, ctype, opA, opB)
    if why:
        ref_err = np.max(np.abs(C - exact) / np.abs(exact))
        assert ref_err > 1e-3, f"expected the reference defect ({why}) but the reference is right"
        return
    assert Co.tobytes() == np.asfortranarray(C).tobytes(), f"C differs in {np.sum(Co != C)} elements"
