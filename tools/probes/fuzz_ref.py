#!/usr/bin/env python3
"""Randomised LIVE parity sweep: this library against the reference's own build (oracle/_ref,
tests/test_ref_parity.py) on identical device inputs, C compared byte for byte.  Random shapes,
type combinations, moduli counts, modes, ops, complex compute types and alpha/beta, minus the
input classes DESIGN.md section 10 lists as reference defects.
python fuzz_ref.py [cases] [seed] [m_n_lo:m_n_hi k_lo:k_hi]
Writes gpurun_out/fuzz_ref.json."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mixed-gemmul8_amd")]
import gemmul8 as G  # noqa: E402
from test_ref_parity import _ref, CODES  # noqa: E402

COMBOS = [("d", "d", "d"), ("s", "s", "s"), ("d", "s", "d"), ("s", "d", "d"), ("d", "s", "s"), ("s", "d", "s"),
          ("z", "z", "z"), ("c", "c", "c"), ("c", "z", "z"), ("z", "c", "z"), ("z", "c", "c"), ("c", "z", "c")]
TDT = {"d": torch.float64, "s": torch.float32, "z": torch.complex128, "c": torch.complex64}
NPT = {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}
MN, K = (1, 600), (1, 1400)


def defect(ta, tb, tc, m, n, k, N, fast, ct, opA, opB, ab):
    """the reference-defect classes of DESIGN.md section 10 (None: a clean case)"""
    cplx = ta in "cz"
    if cplx and ct in (2, 3) and (tc == "z" and N > 7):
        return "10.5"
    if cplx and ct in (2, 3) and ab != (1.0, 0.0):
        return "10.5"
    if cplx and ct == 1 and fast and N == 20:
        return "10.6"
    if (ta, tb, tc) == ("c", "z", "z") and ct == 1:
        return "10.1"
    if cplx and ct == 1 and k % 4 in (2, 3):
        return "10.14"
    if cplx and not fast and ct == 1:
        if opA == 1 or opB == 1:
            return "10.7/10.11"
        if opA == 2 and m != n:
            return "10.12"
        if m % 512 == 256:
            return "10.9"
    if cplx and not fast and ct in (2, 3):
        if opA == 2:
            return "10.13"
        if m % 1024 == 0:
            return "10.15"
    return None


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 1)
    global MN, K
    if len(sys.argv) > 4:  # size ranges: m, n in [a, b), k in [c, d)
        MN, K = tuple(map(int, sys.argv[3].split(":"))), tuple(map(int, sys.argv[4].split(":")))
    lib = _ref()
    t0 = time.time()
    ran, fails, skipped, unchanged = 0, [], {}, []
    while ran < cases:
        ta, tb, tc = COMBOS[rng.integers(len(COMBOS))]
        cplx = ta in "cz"
        m, n = int(rng.integers(MN[0], MN[1])), int(rng.integers(MN[0], MN[1]))
        k = int(rng.integers(K[0], K[1]))
        N = int(rng.integers(2, 21))
        fast = int(rng.integers(2))
        ct = int(rng.integers(1, 4)) if cplx else 0
        opA, opB = int(rng.integers(3 if cplx else 2)), int(rng.integers(3 if cplx else 2))
        ab = [(1.0, 0.0), (1.0, 1.0), (2.5, 0.0)][rng.integers(3)]
        phi = float(rng.choice([0.5, 1.0, 2.0]))
        why = defect(ta, tb, tc, m, n, k, N, fast, ct, opA, opB, ab)
        if why:
            skipped[why] = skipped.get(why, 0) + 1
            continue
        seed = int(rng.integers(1 << 30))
        A = G.randmat(k, m, TDT[ta], phi, seed) if opA else G.randmat(m, k, TDT[ta], phi, seed)
        B = G.randmat(n, k, TDT[tb], phi, seed + 1) if opB else G.randmat(k, n, TDT[tb], phi, seed + 1)
        C0 = G.randmat(m, n, TDT[tc], 0.5, seed + 2)
        lda, ldb = (k if opA else m), (n if opB else k)
        C_ref, C_new = C0.clone(), C0.clone()
        alpha, beta = np.array([ab[0]], NPT[tc]), np.array([ab[1]], NPT[tc])
        wref = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + 16 * max(A.numel(), B.numel()) + (1 << 20),
                           dtype=torch.uint8, device="cuda")
        rc = lib.ref_gemm(CODES[ta], CODES[tb], CODES[tc], opA, opB, m, n, k, alpha.ctypes.data, A.data_ptr(), lda,
                          B.data_ptr(), ldb, beta.ctypes.data, C_ref.data_ptr(), m, N, fast, ct, wref.data_ptr(), None)
        G.gemm(opA, opB, m, n, k, complex(*ab[:1]) if cplx else ab[0], A, lda, B, ldb,
               complex(ab[1]) if cplx else ab[1], C_new, m, N, bool(fast), G.alloc_work(m, n, k, N, ct), ct)
        torch.cuda.synchronize()
        nbad = int((C_ref.view(torch.uint8) != C_new.view(torch.uint8)).sum())
        desc = dict(types=ta + tb + tc, m=m, n=n, k=k, N=N, fast=fast, ct=ct, op=[opA, opB], alpha=ab[0],
                    beta=ab[1], phi=phi, seed=seed, rc=rc, bytes_differ=nbad)
        if torch.equal(C_new.view(torch.uint8), C0.view(torch.uint8)):  # a call that changed nothing
            unchanged.append(desc)
        ran += 1
        if rc != 0 or nbad:
            fails.append(desc)
            print("FAIL", desc, flush=True)
        if ran % 50 == 0:
            print(f"{ran} cases, {len(fails)} failures, {time.time() - t0:.0f} s", flush=True)
    out = dict(cases=ran, failures=fails, outputs_left_unchanged=unchanged, skipped_defect_classes=skipped, seconds=time.time() - t0)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", os.environ.get("FUZZ_OUT", "fuzz_ref.json")), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{ran} cases, {len(fails)} failures, {len(unchanged)} outputs unchanged, skipped {skipped}, "
          f"{time.time() - t0:.0f} s", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
