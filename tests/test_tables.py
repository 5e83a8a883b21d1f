"""Constant tables (mixed-gemmul8_amd/csrc/oz2_tables.inc) against exact big-integer arithmetic,
following GEMMul8/src/table.hpp:1-826 (see tools/gen_tables.py)."""
import math
import os
import re
import sys
from fractions import Fraction

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_tables as gt  # noqa: E402

P = gt.MODULI


def test_moduli_pairwise_coprime_and_le_256():
    assert len(P) == 20 and max(P) == 256
    for i in range(20):
        for j in range(i + 1, 20):
            assert math.gcd(P[i], P[j]) == 1


def test_generated_header_is_current(tmp_path):
    out = tmp_path / "t.inc"
    gt.main.__globals__["sys"].argv = ["gen_tables.py", str(out)]
    gt.main()
    with open(os.path.join(ROOT, "mixed-gemmul8_amd", "csrc", "oz2_tables.inc")) as f:
        cur = f.read()
    assert out.read_text() == cur, "oz2_tables.inc is stale: run python3 tools/gen_tables.py"


def test_crt_weights_are_crt_basis():
    t = gt.build()
    for N in range(2, 21):
        M = math.prod(P[:N])
        for i in range(N):
            w = gt.crt_weights(N)[i]
            for j in range(N):
                assert w % P[j] == (1 if i == j else 0)
        assert t["M_hi"][N - 2] + t["M_lo"][N - 2] == float(M) + t["M_lo"][N - 2]
        assert t["invM"][N - 2] == float(Fraction(1, M))


def test_hi_lo_split_properties():
    """NMi_2 hi parts are exact and their weighted sum cannot overflow 2^53 scaled (exact C1 accumulation);
    hi + lo approximates N_i M_i to double-double accuracy."""
    t = gt.build()
    for N in range(8, 21):
        w = gt.crt_weights(N)
        his = [int(t["NMi_2"][N - 8][i][0]) for i in range(N)]
        tz = min((h & -h).bit_length() - 1 for h in his)
        assert sum(h * (P[i] - 1) for i, h in enumerate(his)) < (1 << (53 + tz))
        for i in range(N):
            lo = t["NMi_2"][N - 8][i][1]
            err = abs(Fraction(his[i]) + Fraction(lo) - w[i])
            assert err <= Fraction(w[i]) * Fraction(1, 1 << 86)  # the reference pins reach 2^-86.4 (N=15)


def test_barrett_constants_and_exact_mod():
    t = gt.build()
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.integers(-2**31, 2**31, 200000, dtype=np.int64),
                         np.array([-2**31, 2**31 - 1, 0, -1, 1, 255, 256, -256], dtype=np.int64)])
    for i in range(1, 20):
        p, inv = P[i], t["barrett"][i]
        assert inv == (1 << 32) // p - 1
        x = xs.copy()
        q = (x * inv) >> 32  # __mulhi
        r = x - q * p
        r = r - (r >= p) * p
        r = r + (r < 0) * p
        assert np.array_equal(r, np.mod(xs, p)), p


def test_log2M_rules():
    t = gt.build()
    for N in range(2, 21):
        M = math.prod(P[:N])
        exact = math.log2(M - 1) / 2
        assert abs(t["log2M_fast"][N - 2] - (exact - 1.5)) < 1e-5
        assert t["log2M_fast"][N - 2] <= exact - 1.5 + 1e-12
        assert abs(t["log2M_accu"][N - 2] - (exact - 0.5)) < 1e-5


def test_tables_compile_as_c_and_cpp(tmp_path):
    """The same header feeds the C oracle (gcc, C11) and the HIP kernels (C++20): both must parse it."""
    import subprocess
    inc = os.path.join(ROOT, "mixed-gemmul8_amd", "csrc", "oz2_tables.inc")
    src = tmp_path / "t.c"
    src.write_text('#include "%s"\nint oz2_probe(void) { return oz2_p[1] + (int)oz2_M_hi[0]; }\n' % inc)
    subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-Wall", str(src)], check=True)
    subprocess.run(["g++", "-std=c++20", "-fsyntax-only", "-x", "c++", str(src)], check=True)
