#!/usr/bin/env python3
"""Randomised parity sweep (GPU vs CPU oracle, bit-exact via tests/test_gpu_parity.check_full):
random shapes, moduli counts, modes, type combinations and ops.  python fuzz_parity.py [cases] [seed]
(GEMMUL8_PERSISTENT=1 GEMMUL8_PERSISTENT_GRID=16 puts every residue product on the persistent kernel
with many tiles per block)"""
import sys
import time

import numpy as np

sys.path[:0] = ["tests", ".", "mixed-gemmul8_amd"]
from test_gpu_parity import check_full, TYPE_COMBOS, _NPT  # noqa: E402
from util import randmat_np  # noqa: E402

cases = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
t0 = time.time()
fails = 0
for c in range(cases):
    ta, tb, tc = TYPE_COMBOS[rng.integers(len(TYPE_COMBOS))]
    cplx = ta in "cz"
    m, n = int(rng.integers(1, 600)), int(rng.integers(1, 600))
    k = int(rng.integers(1, 1400))
    N = int(rng.integers(2, 21))
    fast = bool(rng.integers(2))
    opA, opB = int(rng.integers(3 if cplx else 2)), int(rng.integers(3 if cplx else 2))
    if cplx and not fast:
        opA, opB = 0, 0  # complex accurate mode: the defect-free op combinations
    if cplx and N > 19:
        N = 19  # big-matrix fast mode with 20 moduli is a reference defect
    phi = float(rng.choice([0.5, 1.0, 2.0]))
    A = randmat_np(rng, k, m, phi, _NPT[ta]) if opA else randmat_np(rng, m, k, phi, _NPT[ta])
    B = randmat_np(rng, n, k, phi, _NPT[tb]) if opB else randmat_np(rng, k, n, phi, _NPT[tb])
    desc = f"{ta}{tb}{tc} m={m} n={n} k={k} N={N} {'fast' if fast else 'accu'} op={opA}{opB} phi={phi}"
    try:
        check_full(A, B, N, fast=fast, opA=opA, opB=opB, out_dtype=_NPT[tc])
    except AssertionError as e:
        fails += 1
        print("FAIL", desc, str(e)[:200], flush=True)
    if (c + 1) % 50 == 0:
        print(f"{c + 1} cases, {fails} failures, {time.time() - t0:.0f} s", flush=True)
print(f"{cases} cases, {fails} failures, {time.time() - t0:.0f} s", flush=True)
sys.exit(1 if fails else 0)
