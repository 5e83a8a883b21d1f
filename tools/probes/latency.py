#!/usr/bin/env python3
"""Per-call latency of small DGEMM emulations: eager without / with the phase-timing events, the
host issue time per call, and a HIP graph of one call replayed (launch overhead removed)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mixed-gemmul8_amd"))
import gemmul8 as G  # noqa: E402

sizes = [int(x) for x in (sys.argv[1:] or ["512", "1024", "2048"])]
REPS = 200
for s in sizes:
    m = n = k = s
    A = G.randmat(m, k, torch.float64, 0.5, 123456)
    B = G.randmat(k, n, torch.float64, 0.5, 123456)
    C = torch.empty((n, m), dtype=torch.float64, device="cuda")
    W = G.alloc_work(m, n, k, 14)

    def call():
        G.gemm(0, 0, m, n, k, 1.0, A, m, B, k, 0.0, C, m, 14, True, W)

    for _ in range(10):
        call()
    torch.cuda.synchronize()
    res = {}
    for tim in (False, True):
        G.timing_enable(tim)
        G.timing_read()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(REPS):
            call()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        G.timing_enable(False)
        ph, calls = G.timing_read()
        res["events" if tim else "eager"] = ((t2 - t0) / REPS * 1e6, (t1 - t0) / REPS * 1e6)
        if tim:
            res["phases_us"] = [round(x / max(calls, 1) * 1e3, 1) for x in ph]
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        call()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=st):
            for _ in range(10):
                call()
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS // 10):
        g.replay()
    torch.cuda.synchronize()
    res["graph"] = (time.perf_counter() - t0) / REPS * 1e6
    At, Bt = A.t(), B.t()  # logical m x k, k x n views for rocBLAS DGEMM
    for _ in range(5):
        torch.matmul(At, Bt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        torch.matmul(At, Bt)
    torch.cuda.synchronize()
    res["dgemm"] = (time.perf_counter() - t0) / REPS * 1e6
    print(f"{s}: rocBLAS DGEMM {res['dgemm']:.1f} us/call ({2 * s**3 / res['dgemm'] / 1e6:.1f} TF), "
          f"eager {res['eager'][0]:.1f} us/call ({2 * s**3 / res['eager'][0] / 1e6:.1f} TF; host issue {res['eager'][1]:.1f}), with events "
          f"{res['events'][0]:.1f} (issue {res['events'][1]:.1f}), phases {res['phases_us']}, graph {res['graph']:.1f} us/call",
          flush=True)
