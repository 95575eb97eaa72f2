#!/bin/bash
# Round 4: c2 decoder evidence at HEAD -- SQ counters of one 131072-block call, FETCH/WRITE of one
# call (tools/traffic_call.py), kernel trace of the full 1 M x 16 KiB call, phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04l}; mkdir -p $O
X="tools/exp_time.py 131072 16384 1"
for PASS in 1 2; do
  if [ $PASS = 1 ]; then C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
  else C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"; fi
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/sq/p$PASS -o sq -- python3 $X > $O/sq_p$PASS.txt 2>&1 \
      || { echo "sq pass $PASS failed"; tail -3 $O/sq_p$PASS.txt; exit 1; }
done
python3 tools/pmc_sum.py $O/sq > $O/sq_counters.txt 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/pmc/$c -o run -- python3 $X > $O/pmc_$c.txt 2>&1 \
      || { tail -3 $O/pmc_$c.txt; exit 1; }
done
python3 tools/traffic_call.py $O/pmc k_order_count $((131072 * 16384)) $O/r04_c2_traffic.json | tee $O/traffic.txt || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- \
    python3 tools/exp_time.py 1048576 16384 3 > $O/trace.txt 2>&1 || { tail $O/trace.txt; exit 1; }
python3 tools/kstats.py $(find $O/trace -name "*kernel_trace.csv" | head -1) | tee $O/kernels.txt | head
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids | tee $O/phase.txt
