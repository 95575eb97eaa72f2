#!/bin/bash
# Round 5: decode parity (TEST_LIB) + c2 A/B of library builds (VARIANTS, tools/build_variants.sh)
# + K2 phase stamps of the profile build (tools/phase_prof.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05g}; mkdir -p $O
OUT=${OUT:-r05g} VARIANTS="${VARIANTS:-head}" bash tools/gpu_r5a.sh || exit 1
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids | tee $O/phase.txt
