#!/bin/bash
# Time each experiment build of libqlzx (tools/exp_time.py), one process per build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
: > gpurun_out/exp/times.txt
for so in "$@"; do
  QLZX_EXPERIMENT=1 QLZX_LIB=gobeansdb_amd/$so timeout -k 10 120 python tools/exp_time.py ${EXP_ARGS:-131072 16384 5} >> gpurun_out/exp/times.txt 2>&1 || { echo "FAIL $so rc=$?" >> gpurun_out/exp/times.txt; break; }
done
cat gpurun_out/exp/times.txt
