"""Kernel statistics (rocprofv3 --stats layout) from a rocpd SQLite database (dev tool).
usage: rocpd_stats.py results.db out.csv"""
import csv
import math
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
agg = {}
for name, dur in con.execute("select name, duration from kernels"):
    agg.setdefault(name, []).append(float(dur))
tot = sum(sum(v) for v in agg.values())
with open(sys.argv[2], "w", newline="") as fh:
    w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        m = sum(v) / len(v)
        sd = math.sqrt(sum((x - m) ** 2 for x in v) / len(v))
        w.writerow([name, len(v), int(sum(v)), m, 100.0 * sum(v) / tot, int(min(v)), int(max(v)), sd])
