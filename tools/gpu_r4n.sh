#!/bin/bash
# Round 4: the whole-GPU encoder for values over 64 KiB (tests, 1/8/50 MiB timing against the
# reference) and the chunk-schedule A/B of the batch decoder.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04n}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_large.py \
    > $O/large_tests.log 2>&1 || { tail -40 $O/large_tests.log; exit 1; }
tail -2 $O/large_tests.log
timeout -k 10 500 python -u tools/bench_large.py --out $O/large.json 2>&1 | grep -v amdgpu.ids || exit 1
[ -n "$NOAB" ] && exit 0
NOSQ=1 REPS=${REPS:-2} OUT=${OUT:-r04n} VARIANTS="${VARIANTS:-v4 c256 c256f64 c256f128 c512f128 c128f64}" bash tools/gpu_r4e.sh
