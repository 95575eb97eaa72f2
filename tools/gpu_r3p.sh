#!/bin/bash
# K2b prefetch issued after the batch decode straight into the registers the next decode reads
# (late: GroupRec as four dword loads) vs before it with a copy (early) vs HEAD (base): parity, c2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03p; mkdir -p $O
QLZX_LIB=gobeansdb_amd/libqlzx_late.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_bytes.py tests/test_gpu_codec.py tests/test_gpu_sample_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for t in base late early; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
