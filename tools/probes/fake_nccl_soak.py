#!/usr/bin/env python3
"""Randomised soak of gemmul8.dist's NCCL branch through tests/fake_nccl.py (tests/dist_soak.py: ranks as threads
on one GPU, random shapes / ranks / modes / orders / transfer delays, bit for bit against the single call).
python tools/probes/fake_nccl_soak.py [cases] [seed]"""
import sys
import time

sys.path[:0] = ["tests", ".", "mixed-gemmul8_amd"]
from dist_soak import soak  # noqa: E402

cases = int(sys.argv[1]) if len(sys.argv) > 1 else 50
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
t0 = time.time()
n, fails = soak(cases, seed, log=lambda s: print(f"{s}, {time.time() - t0:.0f} s", flush=True))
for c, msg in fails:
    print("FAIL", c, msg, flush=True)
print(f"done: {cases} cases, {n} failures, {time.time() - t0:.0f} s")
sys.exit(1 if n else 0)
