#!/bin/bash
# K2 profile: phase stamps (profile build), rocprof kernel stats, SQ counters of the split K2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/kp
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 \
    > gpurun_out/kp/phase.txt 2>&1 || { cat gpurun_out/kp/phase.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/kp/phase.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp/trace -o run -- \
    python3 tools/exp_time.py 262144 16384 3 > gpurun_out/kp/trace.txt 2>&1 || { tail gpurun_out/kp/trace.txt; exit 1; }
find gpurun_out/kp/trace -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -12
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/kp/pmc1 -o run -- python3 tools/exp_time.py 131072 16384 1 > gpurun_out/kp/pmc1.txt 2>&1 || { tail gpurun_out/kp/pmc1.txt; exit 1; }
python3 tools/pmc_sum.py gpurun_out/kp/pmc1
