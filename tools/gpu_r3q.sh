#!/bin/bash
# K2b with two items per lane (128-item batches, ipl2) vs one (base): decode parity incl. corrupt
# streams, then interleaved c2 / c5 timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03q; mkdir -p $O
QLZX_LIB=gobeansdb_amd/libqlzx_ipl2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_decode_bytes.py tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_replay.py tests/test_gpu_solo.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for t in base ipl2; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
