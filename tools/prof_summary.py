#!/usr/bin/env python3
"""Summarise a tools/profile.sh directory: per-kernel average duration (kernel trace) and
per-dispatch average of every collected PMC counter, plus derived MFMA utilisation / clock /
HBM bytes (FETCH_SIZE doubled on gfx950 for wide streaming reads, MI355X_MICROARCH.md)."""
import csv
import glob
import json
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
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 128 SIMDs per XCD
        print(f"   MfmaUtil = {100 * avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.1f}%  "
              f"(busy / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)); mean clock over the dispatch "
              f"= {g / 8 / 1e6:.3g} Mcycles")
    if "FETCH_SIZE" in avg:
        print(f"   HBM read  ~ {2 * avg['FETCH_SIZE'] * 1024 / 1e9:.3f} GB per dispatch (FETCH_SIZE KB x2, gfx950 correction)")
    if "WRITE_SIZE" in avg:
        print(f"   HBM write ~ {avg['WRITE_SIZE'] * 1024 / 1e9:.3f} GB per dispatch")
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        h, m = avg["TCC_HIT_sum"], avg["TCC_MISS_sum"]
        print(f"   L2 hit rate = {100 * h / max(h + m, 1):.1f}%")

# machine-readable form: per-kernel average duration and HBM-side bytes per dispatch
out = {"source": d, "kernels": {}}
for k, v in stats.items():
    out["kernels"].setdefault(k, {})["trace_avg_ms"] = sum(v) / len(v)
    out["kernels"][k]["trace_n"] = len(v)
for kn, cs in ctr.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    e = out["kernels"].setdefault(kn, {})
    e["counters"] = avg
    if "FETCH_SIZE" in avg:
        e["hbm_read_bytes"] = 2 * avg["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in avg:
        e["hbm_write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
        e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
for k, e in out["kernels"].items():
    if k.startswith("oz2::gemm_i8_kernel<0") and "hbm_bytes" in e:  # Epi::RESIDUE, the product kernel
        out["gemm_kernel"] = k
        out["gemm_hbm_bytes_per_launch"] = e["hbm_bytes"]
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
