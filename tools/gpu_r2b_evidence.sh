#!/bin/bash
# Round-2 (second session) evidence for c2 at HEAD: full -m gpu suite, the default bench line,
# its rocprof kernel summary, PMC traffic (FETCH_SIZE / WRITE_SIZE) and K2 SQ counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r2b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 400 python -u bench.py > $O/c2_bench.json 2> $O/c2_bench.err || { tail -20 $O/c2_bench.err; exit 1; }
cat $O/c2_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2prof -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/c2_prof_bench.json 2> $O/c2_prof.err || { tail $O/c2_prof.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- \
      python3 bench.py --blocks 131072 --steps 1 --warmup 0 --no-cpu > $O/pmc_$c.json 2> $O/pmc_$c.err || { tail $O/pmc_$c.err; exit 1; }
done
python3 tools/traffic.py $O 131072 $O/c2_traffic.json && cat $O/c2_traffic.json
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
    --output-format csv -d $O/sq -o run -- python3 tools/exp_time.py 131072 16384 2 > $O/sq.txt 2>&1 || { tail -5 $O/sq.txt; exit 1; }
echo done
