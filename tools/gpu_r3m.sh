#!/bin/bash
# Round 3 checkpoint: full GPU suite, the driver's default bench line, rocprof kernel traces of c2
# decode with and without the record CRC (fused into K2), K1/K2 phase stamps (profile build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r03m}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for crc in 0 1; do
  [ $crc = 1 ] && export QLZX_CRC=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_crc$crc -o trace -- \
      python3 tools/exp_time.py 1048576 16384 3 > $O/prof_crc$crc.txt 2>&1 || { echo trace failed; tail $O/prof_crc$crc.txt; exit 1; }
  grep "GiB/s" $O/prof_crc$crc.txt
  python3 tools/kstats.py $(find $O/prof_crc$crc -name "*kernel_trace.csv" | head -1) k_dec k_order | tee $O/prof_crc${crc}_medians.txt
done
unset QLZX_CRC
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids | tee $O/phase.txt
