#!/bin/bash
# Round 4: SQ counters of the 64 KiB encoder on one input class (ENC_ONE=noisy python tools/enc_prof.py N).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04xs}; mkdir -p $O
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
            "SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  ENC_ONE=${KIND:-noisy} REPS=1 timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $O/pass$i -o run -- \
      python3 tools/enc_prof.py ${EN:-4096} 65536 > $O/pass$i.log 2>&1 || { tail $O/pass$i.log; exit 1; }
done
python3 tools/pmc_sum.py $O
