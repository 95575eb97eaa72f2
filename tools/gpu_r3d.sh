#!/bin/bash
# Kernel trace of c2 decode with the record CRC in k_dec_crc; no-far-load bound on K2b.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
export QLZX_CRC=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sep -o trace -- \
    python3 tools/exp_time.py 1048576 16384 3 > $O/prof_sep.txt 2>&1 || { echo trace failed; tail $O/prof_sep.txt; exit 1; }
grep -v amdgpu.ids $O/prof_sep.txt | grep -v rocprofv3 | grep -v "^[EW]2026"
python3 tools/kstats.py $(find $O/prof_sep -name "*kernel_trace.csv" | head -1) k_dec k_order
unset QLZX_CRC
export QLZX_EXPERIMENT=1
for t in sep nofar sep nofar; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done
