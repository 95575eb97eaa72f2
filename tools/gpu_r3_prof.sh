#!/bin/bash
# Round 3: rocprof kernel trace of c2 decode (exp_time, 1 M x 16 KiB) and SQ counters of one
# 131072-block chunk, for the library in gobeansdb_amd/libqlzx.so (or $LIB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03prof}
LIB=${LIB:-gobeansdb_amd/libqlzx.so}
mkdir -p gpurun_out/$TAG
QLZX_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o trace -- \
    python3 tools/exp_time.py 1048576 16384 3 > gpurun_out/$TAG/exp.txt 2>&1 || { echo trace failed; tail gpurun_out/$TAG/exp.txt; exit 1; }
cat gpurun_out/$TAG/exp.txt | grep -v amdgpu.ids
f=$(find gpurun_out/$TAG -name "*kernel_trace.csv" | head -1)
python3 tools/kstats.py "$f" k_dec k_order
QLZX_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
    --output-format csv -d gpurun_out/$TAG/sq -o sq -- python3 tools/exp_time.py 131072 16384 1 > gpurun_out/$TAG/sq.txt 2>&1 || { echo sq failed; tail gpurun_out/$TAG/sq.txt; exit 1; }
python3 tools/pmc_sum.py gpurun_out/$TAG/sq 2>&1 | head -60
