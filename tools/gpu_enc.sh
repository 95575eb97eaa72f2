#!/bin/bash
# GPU check of the workgroup encoder: its parity tests, then the rest of the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_encode_wg.py \
    > gpurun_out/enc_pytest.txt 2>&1
rc=$?; tail -15 gpurun_out/enc_pytest.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests \
    > gpurun_out/all_pytest.txt 2>&1
rc2=$?; tail -5 gpurun_out/all_pytest.txt
exit $(( rc > rc2 ? rc : rc2 ))
