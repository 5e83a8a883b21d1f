"""Randomised LIVE parity sweep against the reference's own build (test helper, not a test file).

This library and the reference's HIP build (oracle/_ref, compiled from the unmodified /root/reference
sources by oracle/ref/Makefile) run on identical device inputs and C is compared byte for byte.  Random
shapes, type combinations, moduli counts, modes, ops, complex compute types and alpha/beta, minus the input
classes DESIGN.md section 10 lists as reference defects (``defect``).  Used by tests/test_ref_parity.py
(GPU) and by the command-line sweep tools/probes/fuzz_ref.py; ``defect`` is pinned on the CPU by
tests/test_ref_sweep_rules.py."""
import ctypes
import os
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "libgemmul8_ref.so")
CODES = {"d": 0, "s": 1, "z": 2, "c": 3}


def _ref():
    """the reference build's ctypes handle (pytest.skip when oracle/_ref was not built)"""
    if not os.path.exists(REF):
        import pytest
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    lib = ctypes.CDLL(REF)
    p, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    lib.ref_gemm.argtypes = [i, i, i, i, i, sz, sz, sz, p, p, sz, p, sz, p, p, sz, u, i, i, p, p]
    lib.ref_work_size.restype = sz
    lib.ref_work_size.argtypes = [sz, sz, sz, u, i]
    return lib


def _extreme(X, vec_axis, big, tiny, sub):
    """Vectors of a column-major matrix held as a torch tensor overwritten with extreme magnitudes
    (vec_axis 1: the rows of A, X[e, v]; 0: the columns of B, X[v, e]): vector 0 subnormal, 1 alternating
    big / tiny, 2 a single subnormal element, 3 zero, 4 big (its sum of squares overflows), 5 negative zeros
    and one normal element."""
    import torch
    V = X if vec_axis == 1 else X.t()  # V[e, v]: element e of vector v
    V[:, 0] *= sub
    alt = torch.ones(V.shape[0], dtype=V.real.dtype if V.is_complex() else V.dtype, device=V.device)
    alt[0::2] = big
    alt[1::2] = tiny
    V[:, 1] *= alt
    V[:, 2] = 0
    V[V.shape[0] // 2, 2] = sub
    V[:, 3] = 0
    V[:, 4] *= big
    V[:, 5] = -0.0
    V[1, 5] = 0.75
    return X


COMBOS = [("d", "d", "d"), ("s", "s", "s"), ("d", "s", "d"), ("s", "d", "d"), ("d", "s", "s"), ("s", "d", "s"),
          ("z", "z", "z"), ("c", "c", "c"), ("c", "z", "z"), ("z", "c", "z"), ("z", "c", "c"), ("c", "z", "c")]
TDT_NAMES = {"d": "float64", "s": "float32", "z": "complex128", "c": "complex64"}
NPT = {"d": np.float64, "s": np.float32, "z": np.complex128, "c": np.complex64}
MN, K = (1, 600), (1, 1400)  # default size ranges: m, n in [1, 600), k in [1, 1400)


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


def sweep(cases, seed, mn=None, kr=None, extreme=False, ab_mode="basic", ld=False, verbose=True, ref_epi=False):
    """run `cases` random calls through both libraries; returns the summary dict (failures first).
    mn, kr: size ranges [lo, hi) of m, n and of k; extreme: half the cases with extreme / non-finite inputs;
    ab_mode "general": complex and general (alpha, beta) too; ld: padded leading dimensions (not with extreme);
    ref_epi: the library in its reference-epilogue mode (gemmul8.set_epilogue), alpha / beta drawn from
    every kernel class including the non-BLAS ones, beta = 0 with alpha != 1 also with non-finite C"""
    import gemmul8 as G
    prev = G.set_epilogue("reference" if ref_epi else "blas")
    try:
        return _sweep(G, cases, seed, mn or MN, kr or K, extreme, ab_mode, ld, verbose, ref_epi)
    finally:
        G.set_epilogue(prev)


def _sweep(G, cases, seed, MN, K, EXTREME, AB, LD, verbose, ref_epi):
    import torch
    TDT = {t: getattr(torch, name) for t, name in TDT_NAMES.items()}
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

