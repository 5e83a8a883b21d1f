#!/usr/bin/env python3
"""One rank's compute in the no-exchange partitions of cfg3 (16384^3, N = 14), measured on one GPU: the output
block of a 2 x 4 (W = 8) or 2 x 2 / 1 x 2 grid -- all moduli for rows [0, m/R) and columns [0, n/Q) -- as one
gemmul8 call on that sub-problem (its own shifts, slices, products and CRT; no collective in fast mode).
Compare with tools/probes/shard_time.py's slowest rank of the (modulus, column block) partition."""
import json
import sys

import torch

sys.path.insert(0, "mixed-gemmul8_amd")
import gemmul8 as G  # noqa: E402


def main():
    n = k = 16384
    N = 14
    A = G.randmat(n, k, torch.float64, 0.5, 123456)
    B = G.randmat(k, n, torch.float64, 0.5, 123456)
    out = {}
    for R, Q in ((1, 1), (1, 2), (2, 2), (2, 4), (1, 8)):
        mb, nb = n // R, n // Q
        w = G.alloc_work(mb, nb, k, N)
        C = torch.empty((nb, mb), dtype=torch.float64, device="cuda")
        call = lambda: G.gemm(G.OP_N, G.OP_N, mb, nb, k, 1.0, A, n, B, k, 0.0, C, mb, N, True, w)
        for _ in range(2):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        G.timing_enable(True)
        G.timing_read()
        e0.record()
        for _ in range(5):
            call()
        e1.record()
        torch.cuda.synchronize()
        G.timing_enable(False)
        ph, _ = G.timing_read()
        ms = e0.elapsed_time(e1) / 5
        out[f"{R}x{Q}"] = {"block": [mb, nb], "ms": round(ms, 3), "phases_ms": [round(x / 5, 3) for x in ph]}
        print(f"{R}x{Q}: block {mb} x {nb}: {ms:.3f} ms, phases {[round(x / 5, 3) for x in ph]}", flush=True)
        del w, C
        torch.cuda.empty_cache()
    with open("gpurun_out/block_time.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
