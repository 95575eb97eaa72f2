#!/bin/bash
# A/B: record CRC in K1 (workgroup of 64/128/256) vs k_dec_crc (main / side stream); K2b 4 vs 8 bytes per lane.
# Then SQ counters of K1 and K2b on one 131072-block chunk (default build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do for t in main bpl8; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
for r in 1 2; do for t in main side k1c256 k1c64 k1c128; do
  QLZX_CRC=1 QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
bash tools/gpu_r3_sq.sh main
