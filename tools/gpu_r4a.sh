#!/bin/bash
# Round-4 baseline at HEAD: c2 kernel trace (1 M blocks, K1/K2 overlap), one chunk alone (K1 and K2b
# serial), SQ counters of one c2 chunk (two passes), K1/K2b phase stamps (profile build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04a}; mkdir -p $O
LIB=${LIB:-gobeansdb_amd/libqlzx.so}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- \
    python3 tools/exp_time.py 1048576 16384 3 > $O/trace.txt 2>&1 || { echo trace failed; tail $O/trace.txt; exit 1; }
grep "GiB/s" $O/trace.txt
python3 tools/kstats.py $(find $O/trace -name "*kernel_trace.csv" | head -1) k_dec k_order | tee $O/medians.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/alone -o trace -- \
    python3 tools/exp_time.py 131072 16384 3 > $O/alone.txt 2>&1 || { echo alone failed; tail $O/alone.txt; exit 1; }
python3 tools/kstats.py $(find $O/alone -name "*kernel_trace.csv" | head -1) k_dec k_order | tee $O/alone_medians.txt
run() {
  QLZX_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/sq/p$PASS -o sq -- \
      python3 tools/exp_time.py 131072 16384 1 > $O/sq_p$PASS.txt 2>&1 || { echo "pass $PASS failed"; tail -3 $O/sq_p$PASS.txt; exit 1; }
  python3 tools/pmc_sum.py $O/sq/p$PASS 2>&1 | tee -a $O/sq_counters.txt
}
PASS=1 run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
PASS=2 run SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids | tee $O/phase.txt
