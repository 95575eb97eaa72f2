"""Per-kernel dispatch statistics from a rocprofv3 SQLite output (run_results.db; tools only).
usage: python tools/kdb.py RUN_RESULTS.db [SUBSTRING ...]"""
import sqlite3
import statistics
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else cols[0])
d = defaultdict(list)
for k, s, e in db.execute(f"select {name}, start, end from kernels"):
    d[str(k).split("(")[0][:48]].append((e - s) / 1e3)
pats = sys.argv[2:]
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if not pats or any(p in k for p in pats):
        print(f"{k:50s} n={len(v):5d} median_us={statistics.median(v):9.1f} mean_us={statistics.mean(v):9.1f} "
              f"sum_us={sum(v):11.1f}")
