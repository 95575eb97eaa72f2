#!/bin/bash
# One GPU-box session: tests, then a short bench.  Stops at the first GPU fault/timeout.
# usage: bash tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 0 pass, 1 test failures; anything else = stop
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${TAG}_pytest.txt; tail -3 gpurun_out/${TAG}_pytest.txt
ok_rc $rc || exit $rc
timeout -k 10 400 python bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/${TAG}_bench.err; tail -2 gpurun_out/${TAG}_bench.err; cat gpurun_out/${TAG}_bench.json
exit $rc
