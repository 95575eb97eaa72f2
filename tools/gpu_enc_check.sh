#!/bin/bash
# Encoder parity tests + per-class encoder timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/enc
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode_wg.py tests/test_gpu_codec.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/enc/pytest.txt 2>&1
rc=$?; tail -5 gpurun_out/enc/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/enc_prof.py ${ENC_ARGS:-16384 65536} > gpurun_out/enc/enc.txt 2>&1; rc=$?
cat gpurun_out/enc/enc.txt; exit $rc
