"""Median/sum per kernel from a rocprofv3 kernel_trace.csv (tools only).
usage: python tools/kstats.py TRACE.csv [SUBSTRING ...]"""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[2:]
d = defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].split("(")[0][:44]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if not pats or any(p in k for p in pats):
        print(f"{k:46s} n={len(v):4d} median_us={statistics.median(v):9.1f} sum_us={sum(v):10.1f}")
