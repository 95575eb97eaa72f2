#!/bin/bash
# PMC counter passes over a short decode bench (one rocprofv3 run per counter set).
# usage: bash tools/pmc.sh TAG "CTR1 CTR2 ..." ["CTRS pass 2" ...]
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
  i=$((i+1))
  mkdir -p gpurun_out/$TAG/pass$i
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/$TAG/pass$i -o run -- \
      python3 bench.py ${PMC_BENCH_ARGS:---blocks 131072 --steps 1 --warmup 0 --cpu-seconds 0} \
      > gpurun_out/$TAG/pass$i/bench.json 2> gpurun_out/$TAG/pass$i/bench.err || exit $?
done
python3 tools/pmc_sum.py gpurun_out/$TAG
