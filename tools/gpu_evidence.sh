#!/bin/bash
# One parameterised GPU-box driver for every committed profile (replaces the per-round
# tools/gpu_r4*.sh / gpu_r5*.sh scripts; their runs are recorded in DESIGN.md's history).
#
# usage (on the box):  gpurun -- 'bash tools/gpu_evidence.sh STEP [STEP ...]'
#   c2         SQ counters (two passes) + FETCH/WRITE of one 131072-block c2 call, kernel trace of the
#              1 M-block call, K1/K2 phase stamps (profile build)  -> $O/{sq_counters.txt,c2_traffic.json,
#              c2_kernel_stats.txt,phase.txt}
#   c3         FETCH/WRITE of the c3 encoder (65536 x 64 KiB) + its kernel trace -> $O/c3_traffic.json
#   c4c5       c4 replay and c5 mixed: kernel traces and one-call FETCH/WRITE -> $O/{c4,c5}_traffic.json
#   single     single-call evidence over 1024 distinct values per size (latency table, 1/16-thread
#              aggregate of this library and the reference) -> $O/single_call.json, $O/mt.jsonl
#   rehearsal  the c4/c5 legs at N = 1 and as a 2-rank gloo group on one GPU; digests compared
#   bench      the default bench line under rocprofv3 --kernel-trace --stats -> $O/bench.json
#   ab TAG...  parity subset on $TEST_TAG's build, then interleaved c2 timing of the builds
#              gobeansdb_amd/libqlzx_TAG.so (tools/build_variants.sh; "head" = the in-tree library)
# Output goes to gpurun_out/${OUT:-r06}; copy what is judged into profiles/ (r06_*).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r06}; mkdir -p $O
lib() { if [ "$1" = head ]; then echo $PWD/gobeansdb_amd/libqlzx.so; else echo $PWD/gobeansdb_amd/libqlzx_$1.so; fi; }
kstats() { python3 tools/kdb.py $(find $1 -name "*results.db" | head -1) > $2 2>/dev/null || \
           python3 tools/kstats.py $(find $1 -name "*kernel_trace.csv" | head -1) > $2; }

step_c2() {
  local X="tools/exp_time.py 131072 16384 1"
  for PASS in 1 2; do
    if [ $PASS = 1 ]; then C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
    else C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"; fi
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/sq/p$PASS -o sq -- python3 $X > $O/sq_p$PASS.txt 2>&1 \
        || { echo "sq pass $PASS failed"; tail -3 $O/sq_p$PASS.txt; return 1; }
  done
  python3 tools/pmc_sum.py $O/sq > $O/sq_counters.txt 2>&1 || return 1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/pmc/$c -o run -- python3 $X > $O/pmc_$c.txt 2>&1 \
        || { tail -3 $O/pmc_$c.txt; return 1; }
  done
  python3 tools/traffic_call.py $O/pmc k_order_count $((131072 * 16384)) $O/c2_traffic.json | tail -3 || return 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o trace -- \
      python3 tools/exp_time.py 1048576 16384 3 > $O/trace.txt 2>&1 || { tail $O/trace.txt; return 1; }
  kstats $O/trace $O/c2_kernel_stats.txt
  QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 \
      | grep -v amdgpu.ids > $O/phase.txt
  tail -n 3 $O/c2_kernel_stats.txt $O/phase.txt
}

step_c3() {
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/c3pmc/pmc_$c -o run -- \
        python3 bench.py --config c3 --blocks 65536 --steps 1 --warmup 0 --no-cpu > $O/c3pmc_$c.json 2> $O/c3pmc_$c.err \
        || { tail $O/c3pmc_$c.err; return 1; }
  done
  python3 tools/traffic.py $O/c3pmc 65536 $O/c3_traffic.json k_encode_wg > /dev/null || return 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3trace -o trace -- \
      python3 bench.py --config c3 --blocks 262144 --steps 2 --warmup 1 --no-cpu > $O/c3_trace.json 2> $O/c3_trace.err \
      || { tail $O/c3_trace.err; return 1; }
  kstats $O/c3trace $O/c3_kernel_stats.txt
  cat $O/c3_traffic.json; head -n 5 $O/c3_kernel_stats.txt
}

step_c4c5() {
  local C4="tools/bench_replay.py --chunk-mib 1000 --files 2 --steps 2 --no-cpu --pin-records 64 --no-gc"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4trace -o trace -- python3 $C4 \
      > $O/c4_trace.json 2> $O/c4_trace.err || { tail $O/c4_trace.err; return 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/c4pmc/$c -o run -- python3 $C4 \
        > $O/c4_$c.json 2> $O/c4_$c.err || { tail $O/c4_$c.err; return 1; }
  done
  local CB=$(python3 -c "import json; print(json.load(open('$O/c4_FETCH_SIZE.json'))['config']['chunk_bytes'][1])")
  python3 tools/traffic_call.py $O/c4pmc k_rp_scan $CB $O/c4_traffic.json | tee $O/c4_traffic.txt || return 1
  local C5="tools/bench_c5.py --total-gib 4 --round-gib 4 --warmup 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5trace -o trace -- python3 $C5 \
      > $O/c5_trace.json 2> $O/c5_trace.err || { tail $O/c5_trace.err; return 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/c5pmc/$c -o run -- python3 $C5 \
        > $O/c5_$c.json 2> $O/c5_$c.err || { tail $O/c5_$c.err; return 1; }
  done
  local RB=$(python3 -c "import json; print(json.load(open('$O/c5_FETCH_SIZE.json'))['config']['round_out_bytes_mean'])")
  python3 tools/traffic_call.py $O/c5pmc k_order_count $RB $O/c5_traffic.json | tee $O/c5_traffic.txt || return 1
  kstats $O/c4trace $O/c4_kernels.txt
  kstats $O/c5trace $O/c5_kernels.txt
  head -n 8 $O/c4_kernels.txt $O/c5_kernels.txt
}

step_single() {
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_service.py \
      tests/test_gpu_solo.py > $O/single_tests.log 2>&1 || { tail -40 $O/single_tests.log; return 1; }
  tail -2 $O/single_tests.log
  timeout -k 10 400 python -u tools/bench_single.py --calls 1000 --values 1024 --threads 16 --dump $O \
      --out $O/single_call.json 2>&1 | grep -v amdgpu.ids || return 1
  gcc -O2 -pthread -o $O/mt_single tools/mt_single.c -ldl || return 1
  : > $O/mt.jsonl
  for n in 4096 16384 65536; do
    for t in 1 16; do
      timeout -k 10 60 $O/mt_single $PWD/gobeansdb_amd/libqlzx.so $O/values_$n.bin $t 2 | tee -a $O/mt.jsonl || return 1
      timeout -k 10 60 $O/mt_single $PWD/oracle/_ref/libqlzref.so $O/values_$n.bin $t 2 | tee -a $O/mt.jsonl || return 1
    done
  done
  rm -f $O/values_*.bin
}

step_rehearsal() {
  timeout -k 10 400 python3 -u bench.py --blocks 65536 --legs-small --no-cpu --steps 3 --warmup 1 \
      > $O/n1.json 2> $O/n1.err || { echo "N=1 failed"; tail -20 $O/n1.err; return 1; }
  QLZX_BENCH_PG=gloo timeout -k 10 500 python3 -u bench.py --gpus 2 --blocks 65536 --legs-small --no-cpu --steps 3 \
      --warmup 1 > $O/n2.json 2> $O/n2.err || { echo "N=2 failed"; tail -20 $O/n2.err; return 1; }
  python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
a, b = (json.loads(open(f"{o}/{n}.json").read().strip().splitlines()[-1]) for n in ("n1", "n2"))
for leg, key in (("replay", "xor_value_crc32"), ("mixed", "xor_output_crc32")):
    print(leg, a[leg]["digest"][key], b[leg]["digest"][key], "equal" if a[leg]["digest"] == b[leg]["digest"] else "DIFFER")
PY
}

step_bench() {
  timeout -k 10 1000 rocprofv3 --kernel-trace --stats -d $O/bench -o bench -- \
      python3 bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; return 1; }
  kstats $O/bench $O/bench_kernel_stats.txt
  find $O/bench -name "*.db" -size +20M -delete
  tail -c 600 $O/bench.json
}

step_ab() {
  if [ -n "$TEST_TAG" ]; then
    QLZX_LIB=$(lib $TEST_TAG) timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
        ${TESTS:-tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_decode_chunk.py tests/test_gpu_replay.py tests/test_gpu_large.py} \
        > $O/ab_tests.log 2>&1 || { tail -30 $O/ab_tests.log; return 1; }
    tail -1 $O/ab_tests.log
  fi
  : > $O/ab.txt
  for r in $(seq ${AB_REPS:-2}); do
    for t in "$@"; do
      QLZX_LIB=$(lib $t) timeout -k 10 180 python -u tools/exp_time.py ${AB_N:-1048576} ${AB_BS:-16384} 5 2>&1 \
          | grep -v amdgpu.ids | sed "s/^/$t /" >> $O/ab.txt || { cat $O/ab.txt; return 1; }
    done
  done
  cat $O/ab.txt
}

# sqab TAG...: one SQ pass (LDS and issue counters) of a 131,072-block c2 call per build (K1/K2 lines)
step_sqab() {
  : > $O/sqab.txt
  for t in "$@"; do
    QLZX_LIB=$(lib $t) timeout -s KILL 90 rocprofv3 --pmc ${SQ_COUNTERS:-SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES} \
        --output-format csv -d $O/sqab/$t -o sq -- python3 tools/exp_time.py 131072 16384 1 > $O/sqab_$t.txt 2>&1 \
        || { echo "sqab $t failed"; tail -3 $O/sqab_$t.txt; return 1; }
    { echo "== $t"; python3 tools/pmc_sum.py $O/sqab/$t | grep -A9 "k_dec_"; } >> $O/sqab.txt || return 1
  done
  cat $O/sqab.txt
}

# abmix TAG...: c5 (64 GiB of mixed values) and c4 (4 x 4000 MiB) per build, interleaved
step_abmix() {
  : > $O/abmix.txt
  for r in $(seq ${AB_REPS:-1}); do
    for t in "$@"; do
      QLZX_LIB=$(lib $t) timeout -k 10 300 python3 tools/bench_c5.py --total-gib 64 --round-gib 16 > $O/c5_$t.json 2>/dev/null \
          || { echo "c5 $t failed"; return 1; }
      QLZX_LIB=$(lib $t) timeout -k 10 400 python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 2 --no-cpu \
          --pin-records 16 > $O/c4_$t.json 2>/dev/null || { echo "c4 $t failed"; return 1; }
      python3 -c "import json; r=json.load(open('$O/c5_$t.json')); q=json.load(open('$O/c4_$t.json')); print('$t c5', r['value'], 'c4', q['value'])" | tee -a $O/abmix.txt
    done
  done
}

while [ $# -gt 0 ]; do
  s=$1; shift
  case $s in
    ab) step_ab "$@" || exit 1; exit 0 ;;
    abmix) step_abmix "$@" || exit 1; exit 0 ;;
    sqab) step_sqab "$@" || exit 1; exit 0 ;;
    c2|c3|c4c5|single|rehearsal|bench) echo "== $s"; step_$s || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
