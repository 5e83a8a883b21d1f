#!/usr/bin/env python3
"""Mid-size timing: for m = n = k in argv (default 1024 1536 2048 3072 4096), per call of
  - the emulated DGEMM, fast and accurate mode, N = 14: back to back (events over 50 calls) and the reference
    driver's way (host clock around each call + device sync, test_double.cu:422-431), with the phase times;
  - rocBLAS DGEMM (torch.matmul on the column-major operands) the same two ways.
Prints one JSON line per size.  Under rocprofv3 --kernel-trace the kernels of every call are listed too."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.environ.get("SMALL_PKG") or os.path.join(ROOT, "mixed-gemmul8_amd"))
import gemmul8 as G  # noqa: E402


def ev_time(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def sync_time(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    t = 0.0
    for _ in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t += time.perf_counter() - t0
    return t / iters * 1e6


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [1024, 1536, 2048, 3072, 4096]
    N = int(os.environ.get("SMALL_N", "14"))
    for s in sizes:
        m = n = k = s
        A = G.randmat(m, k, torch.float64, 0.5, 123456)
        B = G.randmat(k, n, torch.float64, 0.5, 123456)
        C = torch.empty((n, m), dtype=torch.float64, device="cuda")
        w = G.alloc_work(m, n, k, N)
        out = {"size": s, "N": N}
        fl = 2.0 * m * n * k
        for fast in (True, False):
            call = lambda: G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, w)
            tag = "fast" if fast else "accu"
            ev = ev_time(call)
            sy = sync_time(call)
            ph = [0.0] * 4
            for _ in range(20):
                p = G.gemm(G.OP_N, G.OP_N, m, n, k, 1.0, A, m, B, k, 0.0, C, m, N, fast, w, phase_times=True)
                ph = [a + b / 20e3 for a, b in zip(ph, p)]
            out[tag] = {"us_events": round(ev, 2), "us_sync": round(sy, 2), "TF_events": round(fl / ev * 1e-6, 2),
                        "TF_sync": round(fl / sy * 1e-6, 2), "phases_us": [round(x, 2) for x in ph]}
        At, Bt = A.view(k, m), B.view(n, k)  # column-major storage: C^T = B^T A^T in row-major terms
        dg = lambda: torch.matmul(Bt, At, out=C)
        ev = ev_time(dg)
        sy = sync_time(dg)
        out["dgemm"] = {"us_events": round(ev, 2), "us_sync": round(sy, 2), "TF_events": round(fl / ev * 1e-6, 2),
                        "TF_sync": round(fl / sy * 1e-6, 2)}
        print(json.dumps(out), flush=True)
        del A, B, C, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
