#!/bin/bash
# Ablation timing + SQ instruction counts of experiment builds (QLZX_EXPERIMENT: wrong bytes allowed).
# usage: tools/gpu_abl.sh lib1.so ...  ("default" = in-tree lib)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/abl; mkdir -p gpurun_out/abl
for l in "$@"; do
  if [ "$l" = default ]; then lib=$PWD/gobeansdb_amd/libqlzx.so; else lib=$PWD/$l; fi
  tag=$(basename $l .so)
  QLZX_EXPERIMENT=1 QLZX_LIB=$lib timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids >> gpurun_out/abl/time.txt || { cat gpurun_out/abl/time.txt; exit 1; }
  QLZX_EXPERIMENT=1 QLZX_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM \
    --output-format csv -d gpurun_out/abl/$tag -o run -- python3 tools/exp_time.py 131072 16384 1 > gpurun_out/abl/$tag.txt 2>&1 || { tail gpurun_out/abl/$tag.txt; exit 1; }
  echo "== $tag" >> gpurun_out/abl/pmc.txt
  python3 tools/pmc_sum.py gpurun_out/abl/$tag | grep -A8 "k_dec_split" >> gpurun_out/abl/pmc.txt
done
cat gpurun_out/abl/time.txt gpurun_out/abl/pmc.txt
