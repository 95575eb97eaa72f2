#!/bin/bash
# SQ counters of K1/K2 for QLZX_K2=items and =seq (131072 x 16 KiB text, one chunk).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/seqpmc
for m in items seq; do
  QLZX_K2=$m timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
    --output-format csv -d gpurun_out/seqpmc/$m -o run -- python3 tools/exp_time.py 131072 16384 2 > gpurun_out/seqpmc/$m.txt 2>&1 || { tail -5 gpurun_out/seqpmc/$m.txt; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for m in ("items", "seq"):
    f = glob.glob(f"gpurun_out/seqpmc/{m}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "dec_" not in k: continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in acc.items():
        print(m, k[:40], {c: f"{v:.3g}" for c, v in sorted(d.items())})
PY
