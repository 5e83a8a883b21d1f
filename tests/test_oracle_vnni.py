"""The oracle's AVX-512 VNNI int8 products (the CPU baseline's speed) against its scalar loop and exact int64
arithmetic: identical residues for random int8 slices, ragged k (masked tails) and tiny shapes."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = [256, 255, 253, 251, 247, 241, 239, 233, 229, 227, 223, 217, 211, 199, 197, 193, 191, 181, 179, 173]

CHILD = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from oracle import oracle as O
rng = np.random.default_rng(11)
out = []
for (m, n, k, N) in [(37, 29, 131, 14), (5, 3, 64, 7), (64, 64, 63, 20), (300, 200, 257, 9), (1, 1, 1, 2)]:
    A8 = rng.integers(-128, 128, (N, m, k), dtype=np.int8)
    B8 = rng.integers(-128, 128, (N, n, k), dtype=np.int8)
    out.append(O.residues(A8, B8))
np.savez(sys.argv[2], *out, vnni=np.array([O.vnni()]))
'''


def test_vnni_and_scalar_residues_identical(tmp_path):
    res = {}
    for flag in ("0", "1"):
        f = tmp_path / f"r{flag}.npz"
        subprocess.run([sys.executable, "-c", CHILD, ROOT, str(f)], check=True, env=dict(os.environ, OZ2O_SCALAR=flag))
        res[flag] = np.load(f)
    if not bool(res["0"]["vnni"][0]):
        pytest.skip("no AVX-512 VNNI on this host (both runs took the scalar loop)")
    assert not bool(res["1"]["vnni"][0])
    rng = np.random.default_rng(11)
    for i, (m, n, k, N) in enumerate([(37, 29, 131, 14), (5, 3, 64, 7), (64, 64, 63, 20), (300, 200, 257, 9),
                                      (1, 1, 1, 2)]):
        A8 = rng.integers(-128, 128, (N, m, k), dtype=np.int8)
        B8 = rng.integers(-128, 128, (N, n, k), dtype=np.int8)
        exact = np.stack([((A8[j].astype(np.int64) @ B8[j].astype(np.int64).T) % P[j]).T for j in range(N)])
        assert np.array_equal(res["0"][f"arr_{i}"], exact.astype(np.uint8))
        assert np.array_equal(res["1"][f"arr_{i}"], res["0"][f"arr_{i}"])
