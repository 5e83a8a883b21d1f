"""cfg1 (BASELINE.json configs[0]: SGEMM emulation m=n=k=1024, num_moduli=4, fast mode) in full on the CPU:
the oracle on the reference driver's inputs, bit for bit against the reference's own HIP build.

The fixture (tests/golden/cfg1_A.npz: the input, cfg1_ref.json: the hashes of the reference's C and shifts)
was generated on an MI355X by tests/golden/make_golden_cfg1.py, which runs oracle/_ref (the reference's
unmodified gemmul8.cu) on the inputs of gemmul8.randmat (testing/make_matrix.hpp:8-21, seed 123456)."""
import hashlib
import json
import os
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def _sha(x):
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


@pytest.mark.skipif(not os.path.exists(os.path.join(GOLD, "cfg1_A.npz")), reason="cfg1 fixture not generated")
def test_cfg1_oracle_matches_reference_build():
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    meta = json.load(open(os.path.join(GOLD, "cfg1_ref.json")))
    with np.load(os.path.join(GOLD, "cfg1_A.npz")) as z:
        Arows = z["A_colmajor_as_rows"]  # (k, m) rows = the column-major m x k matrix
    assert _sha(Arows) == meta["sha256_A"]
    A = Arows.T  # column-major 1024 x 1024 (F order)
    t0 = time.perf_counter()
    C, sA, sB = O.gemm(A, A, 4, True, return_sft=True)
    dt = time.perf_counter() - t0
    assert C.dtype == np.float32 and C.shape == (1024, 1024)
    assert _sha(sA) == meta["sha256_sftA_reference"] and _sha(sB) == meta["sha256_sftB_reference"]
    # column-major C bytes == the reference's C bytes
    assert _sha(np.asfortranarray(C).T) == meta["sha256_C_reference"]
    assert meta["sha256_C_gemmul8_amd"] == meta["sha256_C_reference"]
    ref = A.astype(np.float64) @ A.astype(np.float64)
    rel = np.abs(C.astype(np.float64) - ref) / np.abs(ref)
    assert abs(float(rel.max()) - meta["relerr_max_vs_fp64"]) <= 1e-12 * max(1.0, meta["relerr_max_vs_fp64"])
    print(f"cfg1 on the CPU: {dt:.2f} s, relerr max {rel.max():.3e} median {np.median(rel):.3e}")
