#!/bin/bash
# K2b prefetch by LDS DMA (main: separate pointer array, 28 WGs/CU; spmk: pointer array aliasing the
# marker ring, 30 WGs/CU) vs register prefetch (nodma, = HEAD) and the HEAD library; decode parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03k; mkdir -p $O
for t in main spmk; do
QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_bytes.py tests/test_gpu_codec.py tests/test_gpu_sample_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests_$t.log 2>&1 || { tail -30 $O/tests_$t.log; exit 1; }
tail -1 $O/tests_$t.log
done
for r in 1 2; do for t in main spmk nodma head; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
for t in main spmk head; do
  QLZX_CRC=1 QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done
