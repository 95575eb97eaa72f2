#!/bin/bash
# Record-CRC kernel: bank-replicated byte table (b16) vs slicing-by-8 (slice8), main / side stream,
# vs the CRC inside K1 (k1crc).  CRC tests first; kernel trace of b16.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03l; mkdir -p $O
QLZX_LIB=gobeansdb_amd/libqlzx_b16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_replay.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do for t in b16 b16side slice8 slice8side k1crc; do
  QLZX_CRC=1 QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
QLZX_LIB=gobeansdb_amd/libqlzx_b16.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
export QLZX_CRC=1 QLZX_LIB=gobeansdb_amd/libqlzx_b16.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- \
    python3 tools/exp_time.py 1048576 16384 3 > $O/prof.txt 2>&1 || { echo trace failed; tail $O/prof.txt; exit 1; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_trace.csv" | head -1) k_dec k_order
