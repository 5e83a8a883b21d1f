#!/usr/bin/env python3
"""Per-call cost in the drivers' loop (device sync + host clock around each call, native code) against the GPU
time of back-to-back calls (events), for the emulation (fast, N = 14) and hipBLAS DGEMM: the host / launch /
sync share of a small call.  python tools/probes/call_overhead.py [sizes]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.environ.get("SMALL_PKG") or os.path.join(ROOT, "mixed-gemmul8_amd"))
import gemmul8 as G  # noqa: E402


def events(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [256, 512, 1024, 2048]
    for s in sizes:
        A = G.randmat(s, s, torch.float64, 0.5, 1)
        B = G.randmat(s, s, torch.float64, 0.5, 2)
        C = torch.empty((s, s), dtype=torch.float64, device="cuda")
        w = G.alloc_work(s, s, s, 14)
        emu = lambda: G.gemm(G.OP_N, G.OP_N, s, s, s, 1.0, A, s, B, s, 0.0, C, s, 14, True, w)
        ev = events(emu)
        tt, ph = G.time_gemm(G.OP_N, G.OP_N, s, s, s, 1.0, A, s, B, s, 0.0, C, s, 14, True, w, 50)
        tv = G.time_vendor_gemm(s, s, s, A, B, C, 50)
        print(json.dumps({"size": s, "emu_events_us": round(ev, 2), "emu_sync_loop_us": round(tt * 1e6, 2),
                          "emu_phase_sum_us": round(sum(ph) * 1e-3, 2), "dgemm_sync_loop_us": round(tv * 1e6, 2)}),
              flush=True)


if __name__ == "__main__":
    main()
