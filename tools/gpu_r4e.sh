#!/bin/bash
# Round 4: decoder variant A/B (c2, 1 M x 16 KiB, interleaved), SQ counters of one c2 chunk for the
# round-3 pair and the default, v4 phase stamps.  Variants: gobeansdb_amd/libqlzx_<tag>.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04e}; mkdir -p $O
: > $O/ab.txt
for rep in $(seq 1 ${REPS:-2}); do
  for l in ${VARIANTS:-v3 v4 k1v3 m256 k1v3m256 w2k nofar}; do
    lib=gobeansdb_amd/libqlzx_$l.so; [ $l = v4 ] && lib=gobeansdb_amd/libqlzx.so
    [ $l = nofar ] && export QLZX_EXPERIMENT=1
    QLZX_LIB=$PWD/$lib timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt
    [ ${PIPESTATUS[0]} -gt 100 ] && exit 1
    unset QLZX_EXPERIMENT
  done
done
sq() {  # $1 tag, $2 lib
  for PASS in 1 2; do
    if [ $PASS = 1 ]; then C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
    else C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"; fi
    QLZX_LIB=$PWD/$2 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/sq_$1/p$PASS -o sq -- \
        python3 tools/exp_time.py 131072 16384 1 > $O/sq_$1_p$PASS.txt 2>&1 || { echo "sq $1 pass $PASS failed"; tail -3 $O/sq_$1_p$PASS.txt; return 1; }
    python3 tools/pmc_sum.py $O/sq_$1/p$PASS 2>&1 | tee -a $O/sq_counters_$1.txt
  done
}
for l in $CRCV; do  # c2 with the fused record CRC (K2<true>)
  lib=gobeansdb_amd/libqlzx_$l.so; [ $l = v4 ] && lib=gobeansdb_amd/libqlzx.so
  QLZX_CRC=1 QLZX_LIB=$PWD/$lib timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | sed "s/^/crc /" | tee -a $O/ab.txt
done
[ -n "$NOSQ" ] && exit 0
sq v3 gobeansdb_amd/libqlzx_v3.so || exit 1
sq v4 gobeansdb_amd/libqlzx.so || exit 1
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids | tee $O/phase.txt
