#!/bin/bash
# A/B of the record-CRC ordering (c2 + CRC): k_dec_crc on the main stream, K1(c+1) after CRC(c) (crcfirst), side stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
for r in 1 2 3; do for t in main crcfirst crcfirst2k side k1c256; do
  QLZX_CRC=1 QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
QLZX_LIB=gobeansdb_amd/libqlzx_main.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
export QLZX_CRC=1 QLZX_LIB=gobeansdb_amd/libqlzx_crcfirst.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- \
    python3 tools/exp_time.py 1048576 16384 3 > $O/prof.txt 2>&1 || { echo trace failed; tail $O/prof.txt; exit 1; }
python3 tools/kstats.py $(find $O/prof -name "*kernel_trace.csv" | head -1) k_dec k_order
