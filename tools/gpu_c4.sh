#!/bin/bash
# c4: rocprof kernel breakdown of the device-only replay (1000 MiB chunk), then the full
# 4000 MiB run with the CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4/trace -o run -- \
    python3 tools/bench_replay.py --chunk-mib 1000 --files 2 --steps 3 --no-cpu > gpurun_out/c4/trace.json 2> gpurun_out/c4/trace.err || { tail gpurun_out/c4/trace.err; exit 1; }
find gpurun_out/c4/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/c4/kernel_stats.csv \;
cut -d, -f1-5 gpurun_out/c4/kernel_stats.csv | head -20
timeout -k 10 700 python3 -u tools/bench_replay.py > gpurun_out/c4/bench.json 2> gpurun_out/c4/bench.err || { tail gpurun_out/c4/bench.err; exit 1; }
cat gpurun_out/c4/bench.json
