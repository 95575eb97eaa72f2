#!/bin/bash
# Decode parity for the default build, then A/B: K2b bytes per lane (8 vs 4), K1 ring rounds (64 vs 32 B),
# chunk size, record-CRC kernel placement; c2 with and without CRC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_bytes.py tests/test_gpu_codec.py tests/test_gpu_sample_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03f/tests.log 2>&1 || { tail -30 gpurun_out/r03f/tests.log; exit 1; }
tail -2 gpurun_out/r03f/tests.log
for r in 1 2; do for t in main bpl4 side r32 ch64k; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
  QLZX_CRC=1 QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
