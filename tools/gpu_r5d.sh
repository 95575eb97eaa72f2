#!/bin/bash
# Round 5: decode parity + c2 A/B (VARIANTS) + v5 phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05g}; mkdir -p $O
OUT=${OUT:-r05g} VARIANTS="${VARIANTS:-v4 v5}" bash tools/gpu_r5a.sh || exit 1
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase5.py 131072 16384 2>&1 | grep -v amdgpu.ids | tee $O/phase5.txt
