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
from test_ref_parity import _ref, _extreme, CODES  # noqa: E402

COMBOS = [("d", "d", "d"), ("s", "s", "s"), ("d", "s", "d"), ("s", "d", "d"), ("d", "s", "s"), ("s", "d", "s"),
          ("z", "z", "z"), ("c", "c", "c"), ("c", "z", "z"), ("z", "c", "z"), ("z", "c", "c"), ("c", "z", "c")]
TDT = {"d": torch.float64, "s": torch.float32, "z": torch.complex128, "c": torch.complex64}
NPT = {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}
MN, K = (1, 600), (1, 1400)
EXTREME = os.environ.get("FUZZ_EXTREME") == "1"
AB = os.environ.get("FUZZ_AB", "basic")
LD = os.environ.get("FUZZ_LD") == "1"  # padded leading dimensions (not with FUZZ_EXTREME)  # "general": complex and general (alpha, beta) too  # half the cases with extreme / non-finite inputs


def defect(ta, tb, tc, m, n, k, N, fast, ct, opA, opB, ab, ref_epi=False):
    """the reference-defect classes of DESIGN.md section 10 (None: a clean case); ref_epi: the library runs in
    its reference-epilogue mode, which reproduces the 10.3 variants"""
    cplx = ta in "cz"
    al, be = ab
    if al == 1 and be not in (0, 1) and not ref_epi:
        return "10.3 (_1b)"
    if al != 1 and be == 1 and tc in "dz" and not ref_epi:
        return "10.3 (_2_a1)"  # (numM = 2 for most N; kept out wholesale)
    if cplx and ct in (2, 3) and (tc == "z" and N > 7):
        return "10.5"
    if cplx and ct in (2, 3) and (al, be) != (1.0, 0.0):
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


def sweep(cases, seed, mn=None, kr=None, extreme=None, ab_mode=None, ld=None, verbose=True, ref_epi=False):
    """run `cases` random calls through both libraries; returns the summary dict (failures first).
    ref_epi: the library in its reference-epilogue mode (gemmul8.set_epilogue), alpha / beta drawn from
    every kernel class including the non-BLAS ones, beta = 0 with alpha != 1 also with non-finite C"""
    prev = G.set_epilogue("reference" if ref_epi else "blas")
    try:
        return _sweep(cases, seed, mn, kr, extreme, ab_mode, ld, verbose, ref_epi)
    finally:
        G.set_epilogue(prev)


def _sweep(cases, seed, mn, kr, extreme, ab_mode, ld, verbose, ref_epi):
    global MN, K, EXTREME, AB, LD
    MN, K = mn or MN, kr or K
    EXTREME = EXTREME if extreme is None else extreme
    AB = AB if ab_mode is None else ab_mode
    LD = LD if ld is None else ld
    rng = np.random.default_rng(seed)
    lib = _ref()
    t0 = time.time()
    ran, fails, skipped, unchanged, nonfinite_vec = 0, [], {}, [], []
    while ran < cases:
        ta, tb, tc = COMBOS[rng.integers(len(COMBOS))]
        cplx = ta in "cz"
        m, n = int(rng.integers(MN[0], MN[1])), int(rng.integers(MN[0], MN[1]))
        k = int(rng.integers(K[0], K[1]))
        N = int(rng.integers(2, 21))
        fast = int(rng.integers(2))
        ct = int(rng.integers(1, 4)) if cplx else 0
        opA, opB = int(rng.integers(3 if cplx else 2)), int(rng.integers(3 if cplx else 2))
        if AB == "general":  # every BLAS-consistent reference kernel (10.3: _1b and _2_a1 are not)
            pool = [(1.0, 0.0), (1.0, 1.0), (2.5, 0.0), (2.5, 0.5), (2.5, 1.0)]
            if cplx:
                pool += [(1.5 - 0.5j, 0.0), (1.5 - 0.5j, 0.25 + 0.75j), (1.0 + 1.0j, 1.0), (2.5, -0.5j),
                         (0.3 + 1.7j, -1.25 + 0.5j), (0.3 + 1.7j, 0.0), (-0.7 + 0.9j, 1.0)]  # inexact ai * x
            if ref_epi:  # the non-BLAS kernels: _1b (alpha = 1, another beta)
                pool += [(1.0, 0.5), (1.0, -1.75)] + ([(1.0, 0.25 + 0.75j)] if cplx else [])
            ab = pool[rng.integers(len(pool))]
        else:
            ab = [(1.0, 0.0), (1.0, 1.0), (2.5, 0.0)][rng.integers(3)]
        phi = float(rng.choice([0.5, 1.0, 2.0]))
        why = defect(ta, tb, tc, m, n, k, N, fast, ct, opA, opB, ab, ref_epi)
        if why:
            skipped[why] = skipped.get(why, 0) + 1
            continue
        seed = int(rng.integers(1 << 30))
        def pad_ld(base):  # FUZZ_LD: leading dimensions beyond the minimum, a fifth of them multiples of 1024
            if not LD:
                return base
            if rng.random() < 0.2:
                return max(1024, (base + 1023) // 1024 * 1024)
            return base + int(rng.integers(0, 41))
        lda, ldb, ldc = pad_ld(k if opA else m), pad_ld(n if opB else k), pad_ld(m)
        # (not only with FUZZ_LD: the minimal leading dimension n or m is itself a multiple of 1024 at large sizes)
        if ldb % 1024 == 0 and opB:
            skipped["10.10"] = skipped.get("10.10", 0) + 1
            continue
        if cplx and lda % 1024 == 0 and not opA:
            skipped["10.17"] = skipped.get("10.17", 0) + 1
            continue
        A = G.randmat(lda, m if opA else k, TDT[ta], phi, seed)
        B = G.randmat(ldb, k if opB else n, TDT[tb], phi, seed + 1)
        special = EXTREME and not LD and rng.random() < 0.5
        inj = []
        if special and ab[0] != 1 and ab[1] == 0 and not ref_epi:  # the reference's _ab reads C at beta = 0
            skipped["10.16"] = skipped.get("10.16", 0) + 1
            continue
        if special:  # extreme vectors (test_ref_parity._extreme) and scattered NaN / +-Inf
            dbl = lambda t: t in "dz"
            for X, t, axis, nv in ((A, ta, 0 if opA else 1, m), (B, tb, 1 if opB else 0, n)):
                if nv >= 6 and X.shape[0] >= 2 and X.shape[1] >= 2:
                    _extreme(X, axis, *((1e200, 1e-200, 1e-310) if dbl(t) else (1e25, 1e-25, 1e-40)))
                for _ in range(int(rng.integers(0, 3))):
                    i, j, val = int(rng.integers(X.shape[0])), int(rng.integers(X.shape[1])), float(
                        rng.choice([np.nan, np.inf, -np.inf]))
                    X[i, j] = val
                    inj.append(["A" if X is A else "B", i, j, str(val)])
        C0 = G.randmat(ldc, n, TDT[tc], 0.5, seed + 2)
        C_ref, C_new = C0.clone(), C0.clone()
        alpha, beta = np.array([ab[0]], NPT[tc]), np.array([ab[1]], NPT[tc])
        if not cplx and (np.iscomplexobj(np.array(ab[0])) or np.iscomplexobj(np.array(ab[1]))):
            continue
        wref = torch.zeros(lib.ref_work_size(m, n, k, N, ct) + 16 * max(A.numel(), B.numel()) + (1 << 20),
                           dtype=torch.uint8, device="cuda")
        rc = lib.ref_gemm(CODES[ta], CODES[tb], CODES[tc], opA, opB, m, n, k, alpha.ctypes.data, A.data_ptr(), lda,
                          B.data_ptr(), ldb, beta.ctypes.data, C_ref.data_ptr(), ldc, N, fast, ct, wref.data_ptr(), None)
        G.gemm(opA, opB, m, n, k, complex(ab[0]) if cplx else ab[0], A, lda, B, ldb,
               complex(ab[1]) if cplx else ab[1], C_new, ldc, N, bool(fast), G.alloc_work(m, n, k, N, ct), ct)
        torch.cuda.synchronize()
        nbad = int((C_ref.view(torch.uint8) != C_new.view(torch.uint8)).sum())
        nonfinite_only = False
        if nbad and special:
            # NaN payload / sign bits are not compared; the rest must lie in rows of op(A) / columns of
            # op(B) that hold a non-finite input (whose shifts the reference derives from Inf / NaN)
            R = torch.view_as_real(C_ref) if cplx else C_ref
            Wn = torch.view_as_real(C_new) if cplx else C_new
            mask = (R.view(torch.uint8).view(R.shape + (-1,)) != Wn.view(torch.uint8).view(Wn.shape + (-1,))).any(-1)
            mask &= ~(torch.isnan(R) & torch.isnan(Wn))
            if cplx:
                mask = mask.any(-1)
            badA = ~torch.isfinite(A).all(dim=1 if opA else 0)  # rows of op(A)
            badB = ~torch.isfinite(B).all(dim=0 if opB else 1)  # columns of op(B)
            inside = badB[:, None] | badA[None, :]  # C is held (n, m)
            nbad = int(mask.sum())
            nonfinite_only = nbad > 0 and bool((mask & ~inside).sum() == 0)
            if nonfinite_only:
                nonfinite_vec.append(int(nbad))
                nbad = 0
        desc = dict(special=bool(special), inj=inj, ld=[lda, ldb, ldc], types=ta + tb + tc, m=m, n=n, k=k, N=N, fast=fast, ct=ct, op=[opA, opB], alpha=str(ab[0]),
                    beta=str(ab[1]), phi=phi, seed=seed, rc=rc, bytes_differ=nbad)
        if torch.equal(C_new.view(torch.uint8), C0.view(torch.uint8)):  # a call that changed nothing
            unchanged.append(desc)
        ran += 1
        if rc != 0 or nbad:
            fails.append(desc)
            if verbose:
                print("FAIL", desc, flush=True)
        if verbose and ran % 50 == 0:
            print(f"{ran} cases, {len(fails)} failures, {time.time() - t0:.0f} s", flush=True)
    return dict(cases=ran, failures=fails, differ_only_in_nonfinite_vectors=len(nonfinite_vec),
                outputs_left_unchanged=unchanged, skipped_defect_classes=skipped, seconds=time.time() - t0)


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    mn = kr = None
    if len(sys.argv) > 4:  # size ranges: m, n in [a, b), k in [c, d)
        mn, kr = tuple(map(int, sys.argv[3].split(":"))), tuple(map(int, sys.argv[4].split(":")))
    t0 = time.time()
    out = sweep(cases, seed, mn, kr, ref_epi=os.environ.get("FUZZ_REF_EPI") == "1")
    ran, fails, skipped = out["cases"], out["failures"], out["skipped_defect_classes"]
    unchanged, nonfinite_vec = out["outputs_left_unchanged"], [0] * out["differ_only_in_nonfinite_vectors"]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", os.environ.get("FUZZ_OUT", "fuzz_ref.json")), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{ran} cases, {len(fails)} failures, {len(unchanged)} outputs unchanged, {len(nonfinite_vec)} differ only in rows / columns with non-finite inputs, skipped {skipped}, "
          f"{time.time() - t0:.0f} s", flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
