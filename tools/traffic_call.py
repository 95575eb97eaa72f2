"""HBM traffic of ONE host call (every kernel it dispatches) from rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes: the dispatches from the last dispatch of FIRST_KERNEL (the call's first kernel)
to the end of the run, per pass (tools only).

usage: python tools/traffic_call.py gpurun_out/TAG FIRST_KERNEL CALL_BYTES OUT.json
Host<->device copies (__amd_rocclr_copyBuffer: the end-to-end leg's pinned D2H) are not part of a
device-resident call and are left out.
  c4: FIRST_KERNEL k_rp_scan (replay index), CALL_BYTES = chunk bytes of that replay
  c5: FIRST_KERNEL k_order_count (batch decompress), CALL_BYTES = decompressed bytes of the round
FETCH_SIZE / WRITE_SIZE are KiB per dispatch; FETCH_SIZE is doubled per MI355X_MICROARCH.md (HBM
section: gfx950 counts half the bytes of 16-B-per-lane streaming reads), WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, first, call_bytes, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
res = {"first_kernel": first, "call_bytes": call_bytes, "kernels": {}, "hbm_bytes_per_call": 0.0}
for counter, scale in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
    rows = []
    for f in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if r["Counter_Name"] == counter]
    disp = defaultdict(float)
    name = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        disp[d] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
    starts = [d for d, n in name.items() if first in n]
    if not starts:
        raise SystemExit(f"{counter}: no dispatch of {first}")
    d0 = max(starts)
    for d in sorted(disp):
        if d < d0 or "copyBuffer" in name[d]:
            continue
        k = name[d].split("(")[0].replace("void ", "")
        e = res["kernels"].setdefault(k, {"dispatches": 0})
        b = scale * 1024 * disp[d]
        e[counter.lower() + "_bytes"] = e.get(counter.lower() + "_bytes", 0.0) + b
        if counter == "FETCH_SIZE":
            e["dispatches"] += 1
        res["hbm_bytes_per_call"] += b
res["hbm_bytes_per_call_byte"] = res["hbm_bytes_per_call"] / call_bytes
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))
for k, v in sorted(res["kernels"].items(), key=lambda kv: -kv[1].get("fetch_size_bytes", 0)):
    print(f"  {k:60s} {v}")
