"""The live sweep's reference-defect classifier (tests/ref_sweep.py ``defect``) on the CPU: every class of
DESIGN.md section 10 that the sweep skips is recognised, and the clean cases around each one are not, so an
edit of the classifier cannot silently widen what the GPU parity test (test_ref_parity.py) leaves out."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ref_sweep import COMBOS, defect  # noqa: E402

CLEAN = (1.0, 0.0)


def d(ta, tb, tc, m=100, n=90, k=64, N=8, fast=1, ct=0, opA=0, opB=0, ab=CLEAN, ref_epi=False):
    return defect(ta, tb, tc, m, n, k, N, fast, ct, opA, opB, ab, ref_epi)


def test_clean_cases_are_not_skipped():
    for ta, tb, tc in COMBOS:
        cplx = ta in "cz"
        for ct in ((1, 2, 3) if cplx else (0,)):
            for fast in (0, 1):
                assert d(ta, tb, tc, k=64, N=6, fast=fast, ct=ct) is None or (ta, tb, tc, ct) == ("c", "z", "z", 1)


def test_epilogue_variants_10_3():
    assert d("d", "d", "d", ab=(1.0, 0.5)) == "10.3 (_1b)"
    assert d("d", "d", "d", ab=(2.5, 1.0)) == "10.3 (_2_a1)"
    assert d("s", "s", "s", ab=(2.5, 1.0)) is None  # float output: one moduli level, BLAS-correct kernel
    assert d("d", "d", "d", ab=(1.0, 0.5), ref_epi=True) is None  # the reference-epilogue mode reproduces them
    assert d("d", "d", "d", ab=(2.5, 0.0)) is None and d("d", "d", "d", ab=(1.0, 1.0)) is None


def test_complex_classes():
    assert d("z", "z", "z", N=8, ct=2) == "10.5" and d("z", "z", "z", N=7, ct=3) is None
    assert d("c", "c", "c", ct=3, ab=(2.5, 0.0)) == "10.5"
    assert d("z", "z", "z", N=20, ct=1) == "10.6" and d("z", "z", "z", N=20, ct=1, fast=0) is None
    assert d("c", "z", "z", ct=1) == "10.1" and d("c", "z", "z", N=6, ct=3) is None
    for k, bad in ((64, False), (65, False), (66, True), (67, True)):
        assert (d("z", "z", "z", k=k, ct=1) == "10.14") == bad
    assert d("z", "z", "z", k=66, N=6, ct=3) is None  # Karatsuba / classic encode the tail correctly


def test_complex_accurate_classes():
    acc = dict(fast=0, ct=1)
    assert d("z", "z", "z", opA=1, **acc) == "10.7/10.11" and d("z", "z", "z", opB=1, **acc) == "10.7/10.11"
    assert d("z", "z", "z", opA=2, m=100, n=90, **acc) == "10.12"
    assert d("z", "z", "z", opA=2, m=90, n=90, **acc) is None
    assert d("z", "z", "z", m=256, **acc) == "10.9" and d("z", "z", "z", m=512, **acc) is None
    assert d("c", "c", "c", fast=0, ct=3, opA=2) == "10.13"
    assert d("c", "c", "c", fast=0, ct=2, m=1024) == "10.15" and d("c", "c", "c", fast=1, ct=2, m=1024) is None


def test_real_types_have_no_shape_classes():
    for m in (256, 512, 1024, 3072):
        for opA in (0, 1):
            for opB in (0, 1):
                assert d("d", "d", "d", m=m, n=m, k=m + 2, opA=opA, opB=opB, fast=0) is None
