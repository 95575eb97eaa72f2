#!/bin/bash
# Round 5: c4 (.data replay) and c5 (mixed values) evidence -- kernel traces (rocprofv3
# --kernel-trace --stats) and FETCH_SIZE / WRITE_SIZE of one call (tools/traffic_call.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05k}; mkdir -p $O
C4="tools/bench_replay.py --chunk-mib 1000 --files 2 --steps 2 --no-cpu --pin-records 64"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4trace -o trace -- python3 $C4 \
    > $O/c4_trace.json 2> $O/c4_trace.err || { tail $O/c4_trace.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/c4pmc/$c -o run -- python3 $C4 \
      > $O/c4_$c.json 2> $O/c4_$c.err || { tail $O/c4_$c.err; exit 1; }
done
CB=$(python3 -c "import json; print(json.load(open('$O/c4_FETCH_SIZE.json'))['config']['chunk_bytes'][1])")
python3 tools/traffic_call.py $O/c4pmc k_rp_scan $CB $O/r05_c4_traffic.json | tee $O/c4_traffic.txt || exit 1
C5="tools/bench_c5.py --total-gib 4 --round-gib 4 --warmup 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5trace -o trace -- python3 $C5 \
    > $O/c5_trace.json 2> $O/c5_trace.err || { tail $O/c5_trace.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/c5pmc/$c -o run -- python3 $C5 \
      > $O/c5_$c.json 2> $O/c5_$c.err || { tail $O/c5_$c.err; exit 1; }
done
RB=$(python3 -c "import json; print(json.load(open('$O/c5_FETCH_SIZE.json'))['config']['round_out_bytes_mean'])")
python3 tools/traffic_call.py $O/c5pmc k_order_count $RB $O/r05_c5_traffic.json | tee $O/c5_traffic.txt || exit 1
python3 tools/kstats.py $(find $O/c4trace -name "*kernel_trace.csv" | head -1) > $O/c4_kernels.txt
python3 tools/kstats.py $(find $O/c5trace -name "*kernel_trace.csv" | head -1) > $O/c5_kernels.txt
head -12 $O/c4_kernels.txt $O/c5_kernels.txt
