#!/bin/bash
# SQ instruction/cycle counters of the decode kernels (131072 x 16 KiB text, 2 dispatches each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/kpmc; mkdir -p gpurun_out/kpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM \
    --output-format csv -d gpurun_out/kpmc/p1 -o run -- python3 tools/exp_time.py 131072 16384 1 > gpurun_out/kpmc/p1.txt 2>&1 || { tail gpurun_out/kpmc/p1.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/kpmc/p2 -o run -- python3 tools/exp_time.py 131072 16384 1 > gpurun_out/kpmc/p2.txt 2>&1 || { tail gpurun_out/kpmc/p2.txt; exit 1; }
python3 tools/pmc_sum.py gpurun_out/kpmc | grep -A20 "k_dec_split\|k_dec_parse<false>\|k_dec_blocks"
