#!/bin/bash
# Round 4: chunk schedule A/B on c2 (1 M x 16 KiB) and c5 (64 GiB of mixed values, 16 GiB rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04p}; mkdir -p $O
: > $O/ab.txt
for rep in 1 2; do
  for l in ${VARIANTS:-v4 c128 c256f64 c256f128}; do
    lib=gobeansdb_amd/libqlzx_$l.so; [ $l = v4 ] && lib=gobeansdb_amd/libqlzx.so
    QLZX_LIB=$PWD/$lib timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt
    [ ${PIPESTATUS[0]} -gt 100 ] && exit 1
    QLZX_LIB=$PWD/$lib timeout -k 10 300 python -u tools/bench_c5.py --total-gib 64 --round-gib 16 2>/dev/null \
      | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$l c5', r['value'], 'GiB/s', r['wall_s'], 's')" | tee -a $O/ab.txt
    [ ${PIPESTATUS[0]} -ne 0 ] && exit 1
  done
done
