#!/bin/bash
# SQ counter passes (one chunk of 131072 x 16 KiB) for library variant $1 (libqlzx_$1.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-v2pj}
mkdir -p gpurun_out/sq_$T
run() {
  QLZX_LIB=gobeansdb_amd/libqlzx_$T.so timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/sq_$T/p$PASS -o sq -- \
      python3 tools/exp_time.py 131072 16384 1 > gpurun_out/sq_$T/p$PASS.txt 2>&1 || { echo "pass $PASS failed"; tail -3 gpurun_out/sq_$T/p$PASS.txt; exit 1; }
  python3 tools/pmc_sum.py gpurun_out/sq_$T/p$PASS 2>&1 | grep -A12 "k_dec_bytes\|k_dec_parse"
}
PASS=1 run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
PASS=2 run SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM
