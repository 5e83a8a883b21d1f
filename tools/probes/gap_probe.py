#!/usr/bin/env python3
"""Where the idle time between cfg2 calls comes from (profiles/r04/final4: the bench's phases sum to 6.09-6.11 ms
per call in every run, the step time is 6.1-6.6 ms).  Runs the bench's timed loop (20 calls, 3 warm-ups) several
times with an event on the stream between calls and a host timestamp after each enqueue; prints, per repeat, the
GPU time per call, the largest and summed gaps between one call's end and the next call's start, and how far
ahead of the GPU the host was when it enqueued each call.  python tools/probes/gap_probe.py [repeats]"""
import gc
import sys
import time

import torch

sys.path.insert(0, "mixed-gemmul8_amd")
import gemmul8 as G  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
m = n = k = 8192
N = 14
A = G.randmat(m, k, torch.float64, 0.5, 123456)
B = A
C = torch.empty((n, m), dtype=torch.float64, device="cuda")
W = G.alloc_work(m, n, k, N)
call = lambda: G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, True, W)
for rep in range(reps):
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
    G.timing_enable(True)
    G.timing_read()
    host = []
    t0 = time.perf_counter()
    for i in range(20):
        ev[2 * i].record()
        call()
        ev[2 * i + 1].record()
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    G.timing_enable(False)
    ph, _ = G.timing_read()
    busy = [ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(20)]
    gaps = [ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(19)]
    start = [ev[0].elapsed_time(ev[2 * i]) for i in range(20)]  # GPU start of call i, ms after call 0's start
    lead = [start[i] - 1e3 * (host[i - 1] if i else 0.0) for i in range(20)]  # >0: host enqueued before the GPU got there
    print(f"rep {rep}: wall {wall * 1e3 / 20:.3f} ms/call, GPU busy {sum(busy) / 20:.3f}, phases {sum(ph) / 20:.3f}, "
          f"gaps sum {sum(gaps):.3f} max {max(gaps):.3f} (at call {gaps.index(max(gaps)) + 1}), "
          f"host lead min {min(lead[1:]):.3f} ms, enqueue of all 20 took {host[-1] * 1e3:.2f} ms, "
          f"gc gen counts {gc.get_count()}", flush=True)
