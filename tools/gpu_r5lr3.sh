#!/bin/bash
# Round 5: K1 per-lane ring, c2 interleaved A/B (HEAD, K = 10, 16) and c5 / c4 slices.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05lr3}; mkdir -p $O
for rep in 1 2 3; do for l in libqlzx.so libqlzx_lr10.so libqlzx_lr16.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 120 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt || exit 1
done; done
for l in libqlzx.so libqlzx_lr10.so libqlzx_lr16.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 300 python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 2 --no-cpu --pin-records 16 > $O/c4_$l.json 2>/dev/null || exit 1
  python3 -c "import json; r=json.load(open('$O/c5_$l.json')); q=json.load(open('$O/c4_$l.json')); print('$l c5', r['value'], 'c4', q['value'])" | tee -a $O/ab.txt
done
