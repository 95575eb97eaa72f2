#!/bin/bash
# K2 iteration: codec GPU tests on the default build, timing of the new and the round-1 K2
# (QLZX_K2=items) on 1 M x 16 KiB text, then the phase profile.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/k2
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/k2/pytest.txt 2>&1
rc=$?; tail -15 gpurun_out/k2/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids > gpurun_out/k2/time.txt || { cat gpurun_out/k2/time.txt; exit 1; }
[ -n "$K2_OLD" ] && { QLZX_K2=split timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids >> gpurun_out/k2/time.txt || { cat gpurun_out/k2/time.txt; exit 1; }; }
cat gpurun_out/k2/time.txt
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids | grep "split" > gpurun_out/k2/phase.txt || { cat gpurun_out/k2/phase.txt; exit 1; }
cat gpurun_out/k2/phase.txt
