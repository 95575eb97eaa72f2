#!/bin/bash
# rocprofv3 kernel-trace + stats of a bench run.  usage: bash tools/prof.sh TAG [bench args...]
set -o pipefail
TAG=${1:-p}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- \
    python3 bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
echo "rc=$rc"
find gpurun_out/$TAG -name "*kernel_stats.csv" -exec cat {} \; | head -20
exit $rc
