#!/bin/bash
# Round 4: decoder variants -- decode parity tests (default lib), A/B timing (c2, 1 M x 16 KiB)
# of the round-3 pair (libqlzx_v3.so), the v4 pair (libqlzx.so) and v4 with 8 bytes per lane
# (libqlzx_b8.so), then kernel traces (whole call and one chunk alone) and v4 phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04b}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_decode_bytes.py \
    tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_replay.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
: > $O/ab.txt
for rep in 1 2; do
  for l in v3 v4 b8; do
    lib=gobeansdb_amd/libqlzx_$l.so; [ $l = v4 ] && lib=gobeansdb_amd/libqlzx.so
    QLZX_LIB=$PWD/$lib timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt
    [ ${PIPESTATUS[0]} -gt 100 ] && exit 1
  done
done
for l in v3 v4; do
  lib=gobeansdb_amd/libqlzx.so; [ $l = v3 ] && lib=gobeansdb_amd/libqlzx_v3.so
  QLZX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$l -o trace -- \
      python3 tools/exp_time.py 1048576 16384 3 > $O/trace_$l.txt 2>&1 || { echo trace failed; tail $O/trace_$l.txt; exit 1; }
  python3 tools/kstats.py $(find $O/trace_$l -name "*kernel_trace.csv" | head -1) k_dec k_order | tee $O/medians_$l.txt
  QLZX_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/alone_$l -o trace -- \
      python3 tools/exp_time.py 131072 16384 3 > $O/alone_$l.txt 2>&1 || { echo alone failed; tail $O/alone_$l.txt; exit 1; }
  python3 tools/kstats.py $(find $O/alone_$l -name "*kernel_trace.csv" | head -1) k_dec k_order | tee $O/alone_medians_$l.txt
done
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids | tee $O/phase.txt
