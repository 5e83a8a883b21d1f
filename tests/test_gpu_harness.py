"""GPU: tools/harness.py writes the reference test drivers' CSV files (GEMMul8/testing/test_double.cu)
with the same headers and row labels, and the numbers behave (errors fall with num_moduli)."""
import csv
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_harness_csv_schema(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import harness
    files = harness.main(["d", "accuracy_check", "flops_check", "--sizes", "512", "--ksizes", "512", "--phi", "0.5",
                          "--moduli", "6", "14", "--iters", "2", "--out-dir", str(tmp_path)])
    acc, tim = files
    rows = list(csv.reader(open(acc)))
    assert rows[0] == ["phi", "function", "6", "14", ""]
    labels = [r[1] for r in rows[1:]]
    assert labels == ["DGEMM (k=512)", "OS2-fast (k=512)", "OS2-accu (k=512)"]
    fast = [float(x) for x in rows[2][2:4]]
    assert fast[1] < fast[0] * 1e-3  # 14 moduli far more accurate than 6
    rows = list(csv.reader(open(tim)))
    assert rows[0] == ["phi", "m", "n", "k", "function", "relerr_max", "relerr_med", "TFLOPS", "total_time [sec]",
                       "conv_64f_2_8i", "gpublasGemmEx", "conv_32i_2_8u", "inverse_scaling", ""]
    assert [r[4] for r in rows[1:]] == ["INT8-GEMM", "DGEMM", "OS2-fast-6", "OS2-fast-14", "OS2-accu-6", "OS2-accu-14"]
    for r in rows[3:]:
        assert float(r[7]) > 0 and float(r[8]) > 0


@pytest.mark.parametrize("t,vend,lo,hi", [("dfd", "DGEMM", 6, 14), ("dff", "SGEMM", 3, 8), ("fC", "CGEMM", 3, 8)])
def test_harness_mixed_and_complex_drivers(tmp_path, t, vend, lo, hi):
    """test_mixed_double.cu / test_mixed_float.cu / test_float_complex.cu: same CSV layout, the
    vendor row named after the routine the driver calls, errors falling with num_moduli."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import harness
    acc, tim = harness.main([t, "accuracy_check", "flops_check", "--sizes", "384", "--ksizes", "384", "--phi",
                             "0.5", "--moduli", str(lo), str(hi), "--iters", "2", "--out-dir", str(tmp_path)])
    assert os.path.basename(acc).startswith(f"oz2_results_{t}_accuracy_")
    rows = list(csv.reader(open(acc)))
    assert [r[1] for r in rows[1:]] == [f"{vend} (k=384)", "OS2-fast (k=384)", "OS2-accu (k=384)"]
    # max elementwise relative errors (near-zero entries of C dominate them, the vendor's too)
    for r in rows[2:]:
        e_lo, e_hi = float(r[2]), float(r[3])
        assert e_hi < 1e-3 * e_lo, (t, r)
    rows = list(csv.reader(open(tim)))
    assert [r[4] for r in rows[1:]] == ["INT8-GEMM", vend, f"OS2-fast-{lo}", f"OS2-fast-{hi}", f"OS2-accu-{lo}",
                                        f"OS2-accu-{hi}"]
    for r in rows[3:]:
        assert float(r[7]) > 0 and float(r[8]) > 0
