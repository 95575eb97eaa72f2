#!/bin/bash
# Round 3: the single-call latency path -- its GPU tests, the decode tests it shares code with,
# phase stamps (profile build), the per-call latency table, and a c2 timing (K2b unchanged).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_solo.py tests/test_gpu_codec.py tests/test_gpu_decode_bytes.py \
    -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_solo_tests.log 2>&1 || { tail -30 gpurun_out/r03_solo_tests.log; exit 1; }
tail -3 gpurun_out/r03_solo_tests.log
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/solo_prof.py 200 2>&1 | grep -v amdgpu.ids
[ "$1" = "short" ] && exit 0
timeout -k 10 300 python -u tools/bench_single.py --calls 300 --out gpurun_out/r03_single_call.json > gpurun_out/r03_single.log 2>&1 || { tail -20 gpurun_out/r03_single.log; exit 1; }
cat gpurun_out/r03_single.log
timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 3 2>&1 | grep -v amdgpu.ids
