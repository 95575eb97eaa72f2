#!/bin/bash
# Full GPU tests, then the default c2 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c2
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/c2/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/c2/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py ${C2_ARGS:---cpu-seconds 15} > gpurun_out/c2/bench.json 2> gpurun_out/c2/bench.err || { tail -20 gpurun_out/c2/bench.err; exit 1; }
cat gpurun_out/c2/bench.json
