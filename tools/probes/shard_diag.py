#!/usr/bin/env python3
"""Diagnose a sharded (modulus, column block) mismatch: runs one case through the single call's phase entry
points and through the simulated ranks of tests/test_gpu_phases.py, and compares the workspace state that
every rank assembles (sft0, bound maxima, sftA, sftB) and the output, printing the first differences.
python tools/probes/shard_diag.py types m n k N W fast opA opB"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mixed-gemmul8_amd")]
import gemmul8 as G  # noqa: E402
from gemmul8 import dist as GD  # noqa: E402
from test_gpu_phases import _rand  # noqa: E402

TDT = {"d": torch.float64, "s": torch.float32, "z": torch.complex128, "c": torch.complex64}


def views(work, L, m, n):
    o = lambda off, cnt, dt: work[off:off + cnt * torch.empty((), dtype=dt).element_size()].view(dt).clone()
    return {"sft0A": o(L["offSft0"], m, torch.int16), "sft0B": o(L["offSft0"] + 2 * L["bm_pad"], n, torch.int16),
            "bound": o(L["offBound"], L["bm_pad"] + -(-n // 256) * 256, torch.int32),
            "sftA": o(L["offSftA"], m, torch.int16), "sftB": o(L["offSftB"], n, torch.int16)}


def main():
    t = sys.argv[1]
    m, n, k, N, W, fast, opA, opB = map(int, sys.argv[2:10])
    ta, tb = t[0], t[1]
    cplx = ta in "zc"
    ct = G.COMPLEX_BIG_MATRIX_ENCODE if cplx else G.REAL_DEFAULT
    out_dtype = TDT["z" if cplx and "z" in t else ("d" if "d" in t else ta)]
    A = _rand(k, m, 1, TDT[ta]) if opA == 0 else _rand(m, k, 1, TDT[ta])
    B = _rand(n, k, 2, TDT[tb]) if opB == 0 else _rand(k, n, 2, TDT[tb])
    lda, ldb = (m if opA == 0 else k), (k if opB == 0 else n)
    L = G.layout(m, n, k, N, ct)
    # single call through the phase entry points
    w1 = G.alloc_work(m, n, k, N, ct)
    if not fast:
        G.split_bound(opA, opB, m, n, k, A, lda, B, ldb, N, w1, out_dtype, ct)
    G.split(opA, opB, m, n, k, A, lda, B, ldb, N, bool(fast), w1, out_dtype, 0, N, ct, bound_ready=not fast)
    G.products(m, n, k, N, w1, 0, N, ct)
    ref = torch.empty((n, m), dtype=out_dtype, device="cuda")
    G.recombine(m, n, k, N, 1.0, 0.0, ref, m, w1, ct)
    torch.cuda.synchronize()
    s1 = views(w1, L, m, n)
    # sharded, keeping every rank's ops
    plan = GD.ShardPlan(m, n, N, W)
    ops = [GD.HipShardOps() for _ in range(W)]
    st = [o.prepare(opA, opB, m, n, k, A, lda, B, ldb, N, bool(fast), out_dtype, ct) for o in ops]
    for r in range(W):
        ops[r].stats(st[r], plan.rows[r], plan.cols[r])
    vecs = [ops[r].shift_vectors(st[r]) for r in range(W)]
    for r in range(W):
        (a0, a1), (b0, b1) = plan.rows[r], plan.cols[r]
        for q in range(W):
            if q != r:
                vecs[q][0][a0:a1] = vecs[r][0][a0:a1]
                vecs[q][1][b0:b1] = vecs[r][1][b0:b1]
    if not fast:
        bnd = [ops[r].bound(st[r], plan.cols[r]).clone() for r in range(W)]
        comb = torch.stack(bnd).amax(0)
        for r in range(W):
            st[r]["work"][L["offBound"]:L["offBound"] + 4 * comb.numel()].view(torch.int32).copy_(comb)
    for r in range(W):
        j0, j1 = plan.mods[r]
        if j1 > j0 or not fast:
            ops[r].encode(st[r], j0, j1)
    torch.cuda.synchronize()
    for r in range(W):
        s2 = views(st[r]["work"], L, m, n)
        for key in ("sft0A", "sft0B", "bound", "sftA", "sftB"):
            if fast and key in ("sft0A", "sft0B", "bound"):
                continue
            d = (s1[key] != s2[key]).nonzero().flatten()
            if d.numel():
                i = int(d[0])
                print(f"rank {r} {key}: {d.numel()} differ, first {i}: single {int(s1[key][i])} sharded {int(s2[key][i])}")
    for t_ in range(plan.stages):
        for r in range(W):
            if t_ < len(plan.launches[r]):
                ops[r].products(st[r], *plan.launches[r][t_])
        for r in range(W):
            for dst, j, a, b in plan.sends(r, t_):
                for x, y in zip(ops[r].chunks(st[r], j, a, b), ops[dst].chunks(st[dst], j, a, b)):
                    y.copy_(x)
    out = torch.cat([ops[r].recombine(st[r], *plan.cols[r]) for r in range(W)], 0)
    torch.cuda.synchronize()
    # residue planes of each rank's own columns against the single call's
    R1 = G.residue_planes(w1, m, n, k, N, 0, N, ct)
    for r in range(W):
        c0, c1 = plan.cols[r]
        R2 = G.residue_planes(st[r]["work"], m, n, k, N, 0, N, ct)
        lo, hi = c0 * L["ldr"], c1 * L["ldr"]
        d = (R1[:, lo:hi] != R2[:, lo:hi]).nonzero()
        if d.numel():
            print(f"rank {r} residues: {d.shape[0]} differ, first plane {int(d[0, 0])} byte {int(d[0, 1]) + lo}")
    nbad = int((out.view(torch.uint8) != ref.view(torch.uint8)).sum())
    print("C bytes differing:", nbad)


if __name__ == "__main__":
    main()
