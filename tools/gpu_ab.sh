#!/bin/bash
# A/B timing of decode builds (QLZX_LIB per build, 1 M x 16 KiB), then the codec GPU tests.
# usage: tools/gpu_ab.sh lib1.so lib2.so ...   (paths relative to the repo root)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for l in "$@"; do
  QLZX_LIB=$PWD/$l timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 >> gpurun_out/ab/time.txt 2>&1 || exit $?
done
cat gpurun_out/ab/time.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/ab/pytest.txt; exit $rc
