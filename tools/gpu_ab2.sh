#!/bin/bash
# A/B timing of decode builds on 1 M x 16 KiB text (each lib's round trip is checked first).
# usage: tools/gpu_ab2.sh lib1.so lib2.so ...   (paths relative to the repo root; "default" = in-tree lib)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
: > gpurun_out/ab/time.txt
for l in "$@"; do
  if [ "$l" = default ]; then lib=$PWD/gobeansdb_amd/libqlzx.so; else lib=$PWD/$l; fi
  QLZX_LIB=$lib timeout -k 10 180 python -u tools/exp_time.py ${AB_N:-1048576} ${AB_BS:-16384} 5 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab/time.txt || { cat gpurun_out/ab/time.txt; exit 1; }
done
cat gpurun_out/ab/time.txt
