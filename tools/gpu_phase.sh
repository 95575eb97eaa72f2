#!/bin/bash
# K1/K2 phase stamps from the -DQLZX_PROFILE build (build it first: python gobeansdb_amd/build.py --profile).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ph
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 \
    > gpurun_out/ph/phase.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ph/phase.txt; exit $rc
