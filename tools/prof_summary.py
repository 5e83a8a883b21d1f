#!/usr/bin/env python3
"""Summarise a tools/profile.sh directory: per-kernel average duration (kernel trace) and
per-dispatch average of every collected PMC counter, plus derived MFMA utilisation / clock /
HBM bytes (FETCH_SIZE doubled on gfx950 for wide streaming reads, MI355X_MICROARCH.md)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]


def short(name):
    return name.split("(")[0].replace("void ", "")[:60]


stats = defaultdict(list)
for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        stats[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print("== kernel trace (ms) ==")
for k, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:60s} n={len(v):3d} avg={sum(v)/len(v):9.4f} total={sum(v):9.3f}")

ctr = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    rows = list(csv.DictReader(open(f)))
    per = defaultdict(lambda: defaultdict(float))
    for r in rows:
        per[(r["Dispatch_Id"], short(r["Kernel_Name"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    for (did, kn), cs in per.items():
        for c, v in cs.items():
            ctr[kn][c].append(v)
print("== PMC (per-dispatch averages) ==")
for kn, cs in ctr.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    line = ", ".join(f"{c}={v:.4g}" for c, v in sorted(avg.items()))
    print(f"{kn}: {line}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        g = avg["GRBM_GUI_ACTIVE"]
        print(f"   MfmaUtil = {100 * avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (g * 1024):.1f}%  (busy / (GRBM_GUI_ACTIVE x 1024 SIMDs))")
    if "FETCH_SIZE" in avg:
        print(f"   HBM read  ~ {2 * avg['FETCH_SIZE'] * 1024 / 1e9:.3f} GB per dispatch (FETCH_SIZE KB x2, gfx950 correction)")
    if "WRITE_SIZE" in avg:
        print(f"   HBM write ~ {avg['WRITE_SIZE'] * 1024 / 1e9:.3f} GB per dispatch")
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        h, m = avg["TCC_HIT_sum"], avg["TCC_MISS_sum"]
        print(f"   L2 hit rate = {100 * h / max(h + m, 1):.1f}%")
