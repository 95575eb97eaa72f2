#!/bin/bash
# rocprof kernel durations of the decode with QLZX_K2=items and =seq (262144 x 16 KiB text).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/seqprof
for m in items seq; do
  QLZX_K2=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/seqprof/$m -o run -- \
    python3 tools/exp_time.py 262144 16384 3 > gpurun_out/seqprof/$m.txt 2>&1 || { tail gpurun_out/seqprof/$m.txt; exit 1; }
  f=$(find gpurun_out/seqprof/$m -name "*kernel_trace.csv" | head -1)
  python3 tools/kstats.py $f dec_ order
done
