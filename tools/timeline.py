"""Per-launch timeline of the LAST decode call in a rocprofv3 kernel_trace.csv (tools only):
start/end of every k_order/k_dec_* dispatch relative to the call's first kernel, in us.
usage: python tools/timeline.py TRACE.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"].split("(")[0].replace("qlzx::", "")[:28], int(r["Start_Timestamp"]),
       int(r["End_Timestamp"])) for r in rows if "k_dec_" in r["Kernel_Name"] or "k_order" in r["Kernel_Name"]]
firsts = [j for j, k in enumerate(ks) if k[0].startswith("k_order_count")]
ks = ks[firsts[-1]:] if firsts else ks
t0 = ks[0][1]
for name, a, b in ks:
    print(f"{name:30s} {(a - t0) / 1e3:9.1f} {(b - t0) / 1e3:9.1f} {(b - a) / 1e3:8.1f}")
print(f"span_us {(max(k[2] for k in ks) - t0) / 1e3:.1f}")
