"""Kernel timeline of one call in a rocprofv3 kernel_trace.csv (tools only): calls are cut at each
dispatch of FIRST_KERNEL; prints the kernels of call INDEX (negative: from the end) that ran at
least 20 us or decode, with start/end relative to the call's first kernel, and the call's span.
usage: python tools/call_timeline.py TRACE.csv FIRST_KERNEL INDEX"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first, index = sys.argv[2], int(sys.argv[3])
cuts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"].split("(")[0]]
print(f"{len(cuts)} calls")
k = cuts[index]
end = cuts[cuts.index(k) + 1] if cuts.index(k) + 1 < len(cuts) else len(rows)
t0 = int(rows[k]["Start_Timestamp"])
for r in rows[k:end]:
    a, b = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("qlzx::", "")[:40]
    if b - a >= 20 or "dec_" in name:
        print(f"{a:9.1f} {b:9.1f} {b - a:8.1f} us  {name}  grid {r.get('Grid_Size_X', '')}")
print(f"span {(int(rows[end - 1]['End_Timestamp']) - t0) / 1e3:.1f} us")
