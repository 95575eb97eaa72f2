#!/bin/bash
# Round 5: v5 ring K2 phase stamps (profile build, K1/K2 not overlapped) + SQ counters (no overlap).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05f}; mkdir -p $O
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase5.py 131072 16384 2>&1 | grep -v amdgpu.ids | tee $O/phase5.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
OUT=${OUT:-r05f} LIBS="${LIBS:-novl v4novl}" bash tools/gpu_r5b.sh
