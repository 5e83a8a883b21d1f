#!/usr/bin/env python3
"""A/B of the CRT across moduli counts: python tools/probes/crt_n_ab.py <variant dir> [<variant dir> ...]
(each directory holds a gemmul8/ package with its own libgemmul8_amd.so).  Every variant runs in its own
subprocess, two rounds: DGEMM 8192^3 fast mode at N = 14, 16, 18, 20, SGEMM 8192^3 at N = 16 and complex
(big-matrix products) 2048^3 at N = 16; prints the CRT phase (ms per call over 10 calls) and a hash of C."""
import json
import subprocess
import sys

CHILD = r'''
import sys, json, hashlib, torch
sys.path.insert(0, sys.argv[1])
import gemmul8 as G
out = {}
cases = [("d%d" % N, 8192, N, torch.float64, G.REAL_DEFAULT) for N in (14, 16, 18, 20)]
cases += [("s16", 8192, 16, torch.float32, G.REAL_DEFAULT), ("z16", 2048, 16, torch.complex128, G.COMPLEX_BIG_MATRIX_ENCODE)]
for name, m, N, dt, ct in cases:
    A = G.randmat(m, m, dt, 0.5, 123456)
    B = G.randmat(m, m, dt, 0.5, 654321)
    C = torch.empty((m, m), dtype=dt, device="cuda")
    w = G.alloc_work(m, m, m, N, ct)
    call = lambda: G.gemm(G.OP_N, G.OP_N, m, m, m, 1.0, A, m, B, m, 0.0, C, m, N, True, w, ct)
    for _ in range(2):
        call()
    torch.cuda.synchronize()
    h = hashlib.sha256(C.cpu().numpy().tobytes()).hexdigest()[:16]
    G.timing_enable(True)
    G.timing_read()
    for _ in range(10):
        call()
    torch.cuda.synchronize()
    G.timing_enable(False)
    ph, _ = G.timing_read()
    out[name] = {"crt_ms": round(ph[3] / 10, 4), "hash": h}
    del A, B, C, w
print(json.dumps(out))
'''

res = {}
for rnd in range(2):
    for v in sys.argv[1:]:
        p = subprocess.run([sys.executable, "-c", CHILD, v], capture_output=True, text=True, timeout=600)
        if p.returncode:
            print(v, "failed:", p.stderr[-2000:])
            sys.exit(1)
        r = json.loads(p.stdout.strip().splitlines()[-1])
        res.setdefault(v, []).append(r)
        print(rnd, v, json.dumps(r), flush=True)
names = list(next(iter(res.values()))[0])
print("hash sets:", {n: sorted({r[n]["hash"] for rr in res.values() for r in rr}) for n in names})
