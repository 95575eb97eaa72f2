#!/bin/bash
# c3 (1 M x 64 KiB image-like compress + fused CRC): the bench line and its rocprof summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3
mkdir -p $O
timeout -k 10 600 python -u bench.py --config c3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu > $O/prof_bench.json 2> $O/prof.err || { tail $O/prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/kstats.py $f encode crc
