#!/bin/bash
# Round 5 evidence at HEAD: c2 SQ counters, FETCH/WRITE of one c2 call, kernel trace and phase
# stamps (as tools/gpu_r4l.sh); c3 FETCH/WRITE (tools/gpu_c3pmc.sh); then the default bench line
# under rocprofv3 --kernel-trace --stats (the rocprof summary of the driver's own command).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05f}; mkdir -p $O
X="tools/exp_time.py 131072 16384 1"
if [ -z "$SKIP_C2" ]; then
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
python3 tools/traffic_call.py $O/pmc k_order_count $((131072 * 16384)) $O/r05_c2_traffic.json | tail -3 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- \
    python3 tools/exp_time.py 1048576 16384 3 > $O/trace.txt 2>&1 || { tail $O/trace.txt; exit 1; }
cp $(find $O/trace -name "*kernel_stats.csv" | head -1) $O/r05_c2_decompress_kernel_stats.csv
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids > $O/phase.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/c3pmc/pmc_$c -o run -- \
      python3 bench.py --config c3 --blocks 65536 --steps 1 --warmup 0 --no-cpu > $O/c3pmc_$c.json 2> $O/c3pmc_$c.err || { tail $O/c3pmc_$c.err; exit 1; }
done
python3 tools/traffic.py $O/c3pmc 65536 $O/r05_c3_traffic.json k_encode_wg > /dev/null || exit 1
fi
timeout -k 10 1000 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench -o bench -- \
    python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cp $(find $O/bench -name "*kernel_stats.csv" | head -1) $O/r05_bench_kernel_stats.csv
rm -rf $O/bench/*/ 2>/dev/null; find $O -name "*kernel_trace.csv" -size +20M -delete
tail -c 600 $O/bench.json
