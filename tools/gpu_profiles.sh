#!/bin/bash
# Round profile set: c2 PMC traffic (FETCH_SIZE, WRITE_SIZE passes), c2 bench with that traffic,
# rocprofv3 kernel-trace stats of the c2 bench, and of a c3 compress bench.
# usage: bash tools/gpu_profiles.sh TAG
set -o pipefail
TAG=${1:-r01v2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
PMC_BENCH_ARGS="--blocks 131072 --steps 1 --warmup 0 --no-cpu" bash tools/pmc.sh $TAG/pmc "FETCH_SIZE" "WRITE_SIZE" > $O/pmc.txt 2>&1 || { tail $O/pmc.txt; exit 1; }
python tools/traffic.py $O/pmc 131072 $O/traffic.json > /dev/null || exit 1
timeout -k 10 600 python bench.py --traffic-json $O/traffic.json > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- \
    python3 bench.py --no-cpu --traffic-json $O/traffic.json > $O/prof_c2_bench.json 2> $O/prof_c2_bench.err || { tail $O/prof_c2_bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- \
    python3 bench.py --mode compress --block-size 65536 --blocks 262144 --steps 3 --warmup 1 --no-cpu \
    > $O/prof_c3_bench.json 2> $O/prof_c3_bench.err || { tail $O/prof_c3_bench.err; exit 1; }
find $O/prof_c2 $O/prof_c3 -name "*kernel_stats.csv" | head
