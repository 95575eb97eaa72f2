#!/bin/bash
# Round 3 evidence: replay CRC table A/B (rpb16 vs rps8), c2 PMC traffic of K1 + K2b, c3 rocprof
# kernel trace and PMC traffic at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03o; mkdir -p $O
QLZX_LIB=gobeansdb_amd/libqlzx_rpb16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_replay.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for t in rpb16 rps8; do
  echo "== $t"; QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 300 python -u tools/bench_replay.py --files 2 --steps 4 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print({k: d[k] for k in d if k in ('value','ms_per_step')})" || exit 1
done; done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/c2pmc_$c -o run -- \
      python3 bench.py --blocks 131072 --steps 1 --warmup 0 --no-cpu --no-c3 --no-c4 --no-c5 --no-crc-leg > $O/c2pmc_$c.json 2> $O/c2pmc_$c.err || { tail $O/c2pmc_$c.err; exit 1; }
done
python3 tools/traffic.py $O 131072 $O/r03_c2_traffic.json && cat $O/r03_c2_traffic.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o run -- \
    python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu > $O/c3prof_bench.json 2> $O/c3prof.err || { tail $O/c3prof.err; exit 1; }
cat $O/c3prof_bench.json | head -c 400; echo
python3 tools/kstats.py $(find $O/c3prof -name "*kernel_trace.csv" | head -1) encode crc | tee $O/c3_medians.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/c3pmc_$c -o run -- \
      python3 bench.py --config c3 --blocks 65536 --steps 1 --warmup 0 --no-cpu > $O/c3pmc_$c.json 2> $O/c3pmc_$c.err || { tail $O/c3pmc_$c.err; exit 1; }
done
python3 tools/traffic.py $O 65536 $O/r03_c3_traffic.json k_encode_wg && cat $O/r03_c3_traffic.json
