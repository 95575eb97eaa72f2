#!/bin/bash
# Round 3, second session: full GPU suite, the driver's default bench line, the single-call
# latency table, and rocprof kernel traces of c2 decode with and without the fused CRC verify.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
O=gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u tools/bench_single.py --calls 300 --out $O/single_call.json > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
cat $O/single.log
for crc in 0 1; do
  [ $crc = 1 ] && export QLZX_CRC=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_crc$crc -o trace -- \
      python3 tools/exp_time.py 1048576 16384 3 > $O/prof_crc$crc.txt 2>&1 || { echo trace failed; tail $O/prof_crc$crc.txt; exit 1; }
  grep -v amdgpu.ids $O/prof_crc$crc.txt
  python3 tools/kstats.py $(find $O/prof_crc$crc -name "*kernel_trace.csv" | head -1) k_dec k_order
done
