#!/bin/bash
# Round 5: where the v5 pair's time goes -- kernel trace of the 1 M-block c2 call and SQ
# counters of one 262144-block call (libraries: LIBS, default the in-tree libqlzx.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05b}; mkdir -p $O
for l in ${LIBS:-v5}; do
  lib=gobeansdb_amd/libqlzx_$l.so; [ $l = head ] && lib=gobeansdb_amd/libqlzx.so
  QLZX_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$l -o kt -- \
      python3 tools/exp_time.py ${NBLK:-1048576} 16384 3 > $O/kt_$l.txt 2>&1 || { echo "kt $l failed"; tail -5 $O/kt_$l.txt; exit 1; }
  f=$(find $O/kt_$l -name "*kernel_trace.csv" | head -1)
  python3 tools/kstats.py $f | tee $O/kstats_$l.txt
  [ -n "$NOSQ" ] && continue
  for PASS in 1 2; do
    if [ $PASS = 1 ]; then C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
    else C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"; fi
    QLZX_LIB=$PWD/$lib timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/sq_$l/p$PASS -o sq -- \
        python3 tools/exp_time.py 262144 16384 1 > $O/sq_${l}_p$PASS.txt 2>&1 || { echo "sq $l pass $PASS failed"; tail -3 $O/sq_${l}_p$PASS.txt; exit 1; }
    python3 tools/pmc_sum.py $O/sq_$l/p$PASS 2>&1 | tee -a $O/sq_counters_$l.txt
  done
done
exit 0
