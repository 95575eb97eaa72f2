#!/bin/bash
# K2 CRC prologue with slicing-by-4 tables (s4) vs the 4-copy byte table (head): decode + CRC
# parity, interleaved c2 timing with the record CRC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ai; mkdir -p $O
QLZX_LIB=gobeansdb_amd/libqlzx_s4.so timeout -k 10 500 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_large.py tests/test_gpu_replay.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in ${REPS:-1 2 3 4}; do for t in ${ORD:-s4 head}; do
  echo -n "crc $t "; QLZX_CRC=1 QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 200 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done; done
echo done
