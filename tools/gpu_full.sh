#!/bin/bash
# Full GPU test suite, then the c3 compress bench (1 M x 64 KiB) with a rocprof kernel summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/full
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/full/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/full/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --mode compress --block-size 65536 --steps 5 --warmup 1 \
    --cpu-seconds 15 > gpurun_out/full/c3.json 2> gpurun_out/full/c3.err || { tail -20 gpurun_out/full/c3.err; exit 1; }
cat gpurun_out/full/c3.json
