#!/bin/bash
# Kernel timeline of one c2 decode call with the record CRC: head (CRC after K1 on K1's stream)
# and c3s (CRC on its own stream), plus the same without the CRC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03v; mkdir -p $O
for t in head c3s; do for crc in 1 0; do
  d=$O/${t}_crc$crc
  if [ $crc = 1 ]; then export QLZX_CRC=1; else unset QLZX_CRC; fi
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- python3 tools/exp_time.py 1048576 16384 3 > $d.log 2>&1 || { tail $d.log; exit 1; }
  echo "== $t crc=$crc"; grep roundtrip $d.log
  python3 tools/timeline.py $(find $d -name "*kernel_trace.csv" | head -1) > $d.timeline.txt && tail -1 $d.timeline.txt
done; done
echo done
