#!/usr/bin/env python3
"""A/B of whole library builds: python tools/probes/lib_ab.py <variant> [<variant> ...]
A variant is a directory holding a gemmul8/ package with its own libgemmul8_amd.so, optionally followed by
@NAME=VALUE,... environment settings for its process (one library, two settings: dir@GEMMUL8_X=0 dir@GEMMUL8_X=1).  Every variant runs in its own
subprocess, alternating over LIB_AB_ROUNDS (default 2) rounds: cfg2 (8192^3, N = 14), cfg5 (complex 4096^3, N = 12, Karatsuba
products) and 8192^2 x 1024 (16 k-steps per tile: the epilogue's share is large), 20 timed calls each after
3 warm-ups; prints ms per call, the phase times (scaling, products, CRT) and a hash of C (the variants must
agree bit for bit)."""
import json
import os
import subprocess
import sys

CHILD = r'''
import sys, json, hashlib, torch
sys.path.insert(0, sys.argv[1])
import gemmul8 as G
out = {}
for name, m, k, N, dt, ct in (("cfg2", 8192, 8192, 14, torch.float64, G.REAL_DEFAULT),
                              ("cfg5", 4096, 4096, 12, torch.complex128, G.COMPLEX_BIG_MATRIX_ENCODE),
                              ("k1024", 8192, 1024, 14, torch.float64, G.REAL_DEFAULT)):
    A = G.randmat(m, k, dt, 0.5, 123456)
    B = G.randmat(k, m, dt, 0.5, 654321)
    C = torch.empty((m, m), dtype=dt, device="cuda")
    w = G.alloc_work(m, m, k, N, ct)
    call = lambda: G.gemm(G.OP_N, G.OP_N, m, m, k, 1.0, A, m, B, k, 0.0, C, m, N, True, w, ct)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    h = hashlib.sha256(C.cpu().numpy().tobytes()).hexdigest()[:16]
    G.timing_enable(True)
    G.timing_read()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        call()
    e1.record()
    torch.cuda.synchronize()
    G.timing_enable(False)
    ph, _ = G.timing_read()
    out[name] = {"ms": round(e0.elapsed_time(e1) / 20, 4), "phases": [round(x / 20, 4) for x in ph], "hash": h}
    del A, B, C, w
    torch.cuda.empty_cache()
print(json.dumps(out))
'''


def main():
    res = {}
    for rnd in range(int(os.environ.get("LIB_AB_ROUNDS", "2"))):
        for v in sys.argv[1:]:
            # "dir" or "dir@NAME=VALUE,NAME=VALUE": the variant's library, with environment settings of its own
            path, _, envs = v.partition("@")
            env = dict(os.environ, **dict(x.split("=", 1) for x in envs.split(",") if x))
            r = subprocess.run([sys.executable, "-c", CHILD, path], capture_output=True, text=True, timeout=300, env=env)
            if r.returncode != 0:
                print(v, "failed", r.stderr[-2000:])
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(rnd, v, json.dumps(d), flush=True)
            res.setdefault(v, []).append(d)
    hashes = {}
    for v in res:
        for d in res[v]:
            for k in d:
                hashes.setdefault(k, set()).add(d[k]["hash"])
    print("hash sets per shape (one hash each when the variants agree):", {k: sorted(s) for k, s in hashes.items()})


if __name__ == "__main__":
    main()
