#!/bin/bash
# Round 4: large values (whole-GPU decoder: tests + timing table), full -m gpu suite, c4 replay
# bench (plan/finish replay, sampled oracle pinning) with its kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04d}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_large.py \
    > $O/large_tests.log 2>&1 || { tail -40 $O/large_tests.log; exit 1; }
tail -2 $O/large_tests.log
timeout -k 10 500 python -u tools/bench_large.py --out $O/large.json 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
    > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
