#!/usr/bin/env python3
"""Per-rank compute time of the (modulus, column block) partition, measured on one GPU: every rank of
ShardPlan(m, n, N, W) is replayed in turn through the native sharded entry points (gemmul8.dist.HipShardOps:
gemmul8_shard_stats over its rows / columns, gemmul8_split of its moduli, its gemmul8_products_cols launches,
gemmul8_recombine_cols of its columns), each phase timed with events on the stream, and the exchange volume
per link taken from the plan.  The critical path of a W-GPU run is the slowest rank's compute plus whatever
part of its receives does not overlap (the last stage's); the collectives (one all-gather of m + n int16)
are left out.

    python tools/probes/shard_time.py [size] [N] [W ...]     (defaults: 16384 14 2 4 8)
    SHARD_ORDER=columns: ShardPlan's column-block-major unit order (default moduli)
    SHARD_GRID=2: the 2-D grid of gemmul8.dist.gemm_moduli_grid instead -- H = 2 row blocks of W / 2 ranks, each
    rank replayed as rank (W/2-rank plan) of row block 0's sub-problem (rows [0, m/2) of A; both blocks cost the
    same)"""
import os
import json
import sys

import torch

sys.path.insert(0, "mixed-gemmul8_amd")
import gemmul8 as G  # noqa: E402
from gemmul8 import dist as GD  # noqa: E402


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    Ws = [int(x) for x in sys.argv[3:]] or [2, 4, 8]
    n = k = m
    A = G.randmat(m, k, torch.float64, 0.5, 123456)
    B = G.randmat(k, n, torch.float64, 0.5, 123456)
    ops = GD.HipShardOps()
    st = ops.prepare(G.OP_N, G.OP_N, m, n, k, A, m, B, k, N, True, torch.float64, G.REAL_DEFAULT)
    # the whole call once on this workspace: every shift in place, so each replayed rank encodes real slices
    C = torch.empty((n, m), dtype=torch.float64, device="cuda")
    G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, True, st["work"])
    t_single = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, True, st["work"])
        e1.record()
        torch.cuda.synchronize()
        t_single.append(e0.elapsed_time(e1))
    single = min(t_single)
    out = {"shape": [m, n, k], "N": N, "single_gpu_ms": round(single, 3), "W": {}}
    print(f"single GPU: {single:.3f} ms ({2.0 * m * n * k / single / 1e9:.1f} TFLOP/s)", flush=True)

    def timed(fn, reps=2):
        best = None
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1)
            best = t if best is None else min(best, t)
        return best

    H = int(os.environ.get("SHARD_GRID", "1"))
    sub_st = {}
    for W in Ws:
        Wp, mp, stp = W, m, st
        if H > 1:  # the grid: row block 0's sub-problem over W / H ranks
            Wp, mp = W // H, GD.blocks(m, H)[0][1]
            if mp not in sub_st:
                ops_h = GD.HipShardOps()
                sub_st[mp] = ops_h.prepare(G.OP_N, G.OP_N, mp, n, k, A[:, :mp], m, B, k, N, True, torch.float64,
                                           G.REAL_DEFAULT)
                Ch = torch.empty((n, mp), dtype=torch.float64, device="cuda")
                G.gemm(G.OP_N, G.OP_N, mp, n, k, 1.0, A[:, :mp], m, B, k, 0.0, Ch, mp, N, True, sub_st[mp]["work"])
            stp = sub_st[mp]
        plan = GD.ShardPlan(mp, n, N, Wp, order=os.environ.get("SHARD_ORDER", "moduli"))
        st_w = stp
        ranks = []
        for r in range(Wp):
            st = st_w
            j0, j1 = plan.mods[r]
            c0, c1 = plan.cols[r]
            ph = {"stats": timed(lambda: ops.stats(st, plan.rows[r], plan.cols[r])),
                  "encode": timed(lambda: ops.encode(st, j0, j1)) if j1 > j0 else 0.0,
                  "products": [timed(lambda u=u: ops.products(st, *u)) for u in plan.launches[r]],
                  "crt": timed(lambda: ops.recombine(st, c0, c1))}
            recv = sum((b - a) * mp * (3 if st["L"]["nsub"] == 3 else 1)
                       for t in range(plan.stages) for (_, j, a, b) in plan.recvs(r, t))
            links = {}
            for t in range(plan.stages):
                for (src, j, a, b) in plan.recvs(r, t):
                    links[src] = links.get(src, 0) + (b - a) * mp
            last = plan.recvs(r, plan.stages - 1) if plan.stages else []
            total = ph["stats"] + ph["encode"] + sum(ph["products"]) + ph["crt"]
            ranks.append({"rank": r, "ms": {kk: (round(v, 3) if not isinstance(v, list) else [round(x, 3) for x in v])
                                            for kk, v in ph.items()},
                          "compute_ms": round(total, 3), "recv_bytes": recv,
                          "max_link_bytes": max(links.values()) if links else 0,
                          "last_stage_recv_bytes": sum((b - a) * mp for (_, j, a, b) in last)})
        worst = max(x["compute_ms"] for x in ranks)
        eff = single / (W * worst)
        out["W"][W] = {"ranks": ranks, "slowest_rank_compute_ms": worst,
                       "tflops_compute_only": round(2.0 * m * n * k / worst / 1e9, 1),
                       "efficiency_compute_only": round(eff, 3)}
        print(f"W={W}: slowest rank {worst:.3f} ms compute ({2.0 * m * n * k / worst / 1e9:.1f} TFLOP/s), "
              f"efficiency {eff:.3f}; max link {max(x['max_link_bytes'] for x in ranks) / 1e6:.0f} MB, "
              f"last-stage receive {max(x['last_stage_recv_bytes'] for x in ranks) / 1e6:.0f} MB", flush=True)
        for x in ranks:
            print("   ", json.dumps(x), flush=True)
    with open("gpurun_out/shard_time_%s%s.json" % (os.environ.get("SHARD_ORDER", "moduli"),
                                                  "_grid%d" % H if H > 1 else ""), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
