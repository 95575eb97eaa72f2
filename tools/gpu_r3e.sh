#!/bin/bash
# A/B of the record-CRC kernel placement (fused-CRC c2 decode), plus a kernel trace of the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
#timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_sample_parity.py -x -q --timeout 200 --timeout-method thread -k crc > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
#tail
export QLZX_CRC=1
for r in 1 2; do for t in g1k w512g1k w512g2k g2k g4k sideg2k; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- \
    python3 tools/exp_time.py 1048576 16384 3 > $O/prof.txt 2>&1 || { echo trace failed; tail $O/prof.txt; exit 1; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_trace.csv" | head -1) k_dec k_order
