#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
: > gpurun_out/exp/times.txt
A="${EXP_ARGS:-1048576 16384 5}"
QLZX_LIB=gobeansdb_amd/libqlzx.so timeout -k 10 200 python tools/exp_time.py $A >> gpurun_out/exp/times.txt 2>&1 || exit 1
QLZX_K1_OVERLAP=1 QLZX_LIB=gobeansdb_amd/libqlzx.so timeout -k 10 200 python tools/exp_time.py $A >> gpurun_out/exp/times.txt 2>&1 || exit 1
QLZX_LIB=gobeansdb_amd/libqlzx_r32.so timeout -k 10 200 python tools/exp_time.py $A >> gpurun_out/exp/times.txt 2>&1 || exit 1
QLZX_K1_OVERLAP=1 QLZX_LIB=gobeansdb_amd/libqlzx_r32.so timeout -k 10 200 python tools/exp_time.py $A >> gpurun_out/exp/times.txt 2>&1 || exit 1
cat gpurun_out/exp/times.txt
