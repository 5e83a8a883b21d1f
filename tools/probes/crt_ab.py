#!/usr/bin/env python3
"""A/B of CRT kernel builds: python tools/probes/crt_ab.py <variant dir> [<variant dir> ...]
Each directory holds a gemmul8/ package with its own libgemmul8_amd.so (tools/probes/crt_ab/<v>/).  Every
variant runs in its own subprocess: one full call at the cfg5 shape (complex 4096^3, N = 12, big matrix ->
Karatsuba products) and at cfg2 (8192^3, N = 14), then the recombine phase alone timed with events; prints
ms per CRT and a hash of C (the variants must agree bit for bit)."""
import hashlib
import json
import subprocess
import sys

CHILD = r'''
import sys, json, hashlib, torch
sys.path.insert(0, sys.argv[1])
import gemmul8 as G
out = {}
for name, m, N, dt, ct in (("cfg5", 4096, 12, torch.complex128, G.COMPLEX_BIG_MATRIX_ENCODE),
                           ("cfg2", 8192, 14, torch.float64, G.REAL_DEFAULT)):
    A = G.randmat(m, m, dt, 0.5, 123456)
    C = torch.empty((m, m), dtype=dt, device="cuda")
    w = G.alloc_work(m, m, m, N, ct)
    G.gemm(G.OP_N, G.OP_N, m, m, m, 1.0, A, m, A, m, 0.0, C, m, N, True, w, ct)
    torch.cuda.synchronize()
    h = hashlib.sha256(C.cpu().numpy().tobytes()).hexdigest()[:16]
    for _ in range(3):
        G.recombine(m, m, m, N, 1.0, 0.0, C, m, w, ct)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        G.recombine(m, m, m, N, 1.0, 0.0, C, m, w, ct)
    e1.record()
    torch.cuda.synchronize()
    h2 = hashlib.sha256(C.cpu().numpy().tobytes()).hexdigest()[:16]
    out[name] = {"crt_ms": e0.elapsed_time(e1) / 50, "hash": h, "hash_after": h2}
    del A, C, w
    torch.cuda.empty_cache()
print(json.dumps(out))
'''


def main():
    res = {}
    for rnd in range(2):
        for v in sys.argv[1:]:
            r = subprocess.run([sys.executable, "-c", CHILD, v], capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(v, "failed", r.stderr[-2000:])
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            print(rnd, v, json.dumps(d), flush=True)
            res.setdefault(v, []).append(d)
    hashes = {(k, d[k]["hash"]) for v in res for d in res[v] for k in d}
    print("hashes:", sorted(hashes))


if __name__ == "__main__":
    main()
