#!/bin/bash
# What an instruction costs in K2b: +32 / +64 independent VALU or +32 SALU per 256-B chunk
# (64 chunks per c2 block; the bytes are unchanged), interleaved c2 timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2 3; do for t in base padv32 padv64 pads32; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
