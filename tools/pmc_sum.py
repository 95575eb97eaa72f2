"""Summarise rocprofv3 --pmc counter CSVs: per kernel name, mean of each counter over dispatches."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name", "")
            if "qlzx" not in name:
                continue
            short = name.split("(")[0].replace("void ", "")
            acc[short][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, d in acc.items():
    per = defaultdict(list)
    for (disp, c), v in d.items():
        per[c].append(sum(v))
    print(k)
    for c in sorted(per):
        vals = per[c]
        print(f"   {c:28s} {sum(vals) / len(vals):16.4g}   (dispatches {len(vals)})")
