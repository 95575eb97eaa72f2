#!/bin/bash
# k_dec_seq bring-up: the decode parity tests for every K2 kernel, then c2 timing of
# the default K2 and QLZX_K2=seq (each run checks its round trip first).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/seq
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_large.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/seq/tests.txt 2>&1
rc=$?
tail -25 gpurun_out/seq/tests.txt
[ $rc -eq 0 ] || exit $rc
for m in items seq items seq; do
  QLZX_K2=$m timeout -k 10 180 python -u tools/exp_time.py ${AB_N:-1048576} ${AB_BS:-16384} 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$m /" || exit 1
done
