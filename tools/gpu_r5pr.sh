#!/bin/bash
# Wave priority A/B (s_setprio at K2 entry, then at K1 entry in the second run; libqlzx_p1.so = 1, libqlzx_p3.so = 3, libqlzx.so = 0):
# c2 (tools/exp_time.py), c5 (64 GiB) and c4 (4 x 4000 MiB) interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05pr; mkdir -p $O
for r in 1 2; do
  for l in libqlzx.so libqlzx_p1.so libqlzx_p3.so; do
    echo "== c2 $(QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c5_$l.json')); print('== c5 $l', d['value'])"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 2 --no-cpu > $O/c4_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c4_$l.json')); print('== c4 $l', d['value'])"
  done
done
