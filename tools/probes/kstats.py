#!/usr/bin/env python3
"""Print the average duration of each library kernel in a rocprofv3 kernel_stats.csv
(optionally only names containing a filter word)."""
import csv
import sys

flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "oz2::" in n and flt in n:
        print("   %-62s %5s %9.2f us" % (n[:62], r["Calls"], float(r["AverageNs"]) / 1e3))
