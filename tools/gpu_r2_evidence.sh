#!/bin/bash
# Round-2 evidence: default c2 bench line (with the CPU leg), its rocprof kernel summary,
# the c3 bench line and its rocprof summary, single-call latency, and c2 PMC traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r2e
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || { tail -20 $O/c2_bench.err; exit 1; }
cat $O/c2_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2prof -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/c2_prof_bench.json 2> $O/c2_prof.err || { tail $O/c2_prof.err; exit 1; }
timeout -k 10 500 python -u bench.py --config c3 > $O/c3_bench.json 2> $O/c3_bench.err || { tail -20 $O/c3_bench.err; exit 1; }
cat $O/c3_bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o run -- \
    python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu > $O/c3_prof_bench.json 2> $O/c3_prof.err || { tail $O/c3_prof.err; exit 1; }
timeout -k 10 300 python -u tools/bench_single.py --calls 200 --out $O/single.json > $O/single.txt 2>&1 || { tail $O/single.txt; exit 1; }
cat $O/single.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- \
      python3 bench.py --blocks 131072 --steps 1 --warmup 0 --no-cpu > $O/pmc_$c.json 2> $O/pmc_$c.err || { tail $O/pmc_$c.err; exit 1; }
done
python3 tools/traffic.py $O 131072 $O/c2_traffic.json && cat $O/c2_traffic.json
