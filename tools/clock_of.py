#!/usr/bin/env python3
"""clock_of.py <counter_collection.csv> -- per kernel: average duration, effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / duration) and MFMA busy fraction, from a rocprofv3 --pmc pass
with GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES."""
import csv
import sys
from collections import defaultdict

rows = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:70]
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows[k][r["Counter_Name"]].append((float(r["Counter_Value"]), d))
for k, c in rows.items():
    g = c.get("GRBM_GUI_ACTIVE")
    if not g:
        continue
    dur = sum(d for _, d in g) / len(g)
    clk = sum(v for v, _ in g) / len(g) / 8 / dur
    line = f"{k:70s} n={len(g):3d} {dur / 1e6:8.3f} ms  clk {clk:5.2f} GHz"
    m = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
    if m:
        # MFMA busy cycles are summed over 256 CUs (x4 SIMDs) -- ratio against GRBM cycles per CU
        mb = sum(v for v, _ in m) / len(m)
        line += f"  mfma_busy/cu/clk {mb / 256 / (clk * dur):6.3f}"
    print(line)

# every other counter of the pass, per CU per (GRBM) cycle
for k, c in rows.items():
    g = c.get("GRBM_GUI_ACTIVE")
    if not g or not any(w in k for w in ("gemm", "encode", "stats", "crt")):
        continue
    cyc = sum(v for v, _ in g) / len(g) / 8
    for name, vals in c.items():
        if name in ("GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"):
            continue
        v = sum(x for x, _ in vals) / len(vals)
        print(f"    {name:40s} {v:14.4g}  per CU per cycle {v / 256 / cyc:8.4f}")
