#!/bin/bash
# FETCH_SIZE calibration (tools/mb/mb_fetch.hip): counter value per kernel vs the known 512 MiB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/fetchcal
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fetchcal -o run -- ./tools/mb/mb_fetch > gpurun_out/fetchcal/out.txt 2>&1 || { tail gpurun_out/fetchcal/out.txt; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/fetchcal/**/*counter_collection.csv", recursive=True)[0]
tot = collections.OrderedDict()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0] + "#" + r["Dispatch_Id"]
    tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
true_kib = 512 * 1024
for k, v in tot.items():
    print(f"{k:40s} FETCH_SIZE {v:12.0f} KiB  counted/true {v / true_kib:.3f}  correction x{true_kib / v:.3f}")
PY
