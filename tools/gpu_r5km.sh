#!/bin/bash
# K1 step budget under the iterative-ILP build: uniform calls 12 / 20 (libqlzx_u12/u20.so) and mixed
# calls 8 / 12 (libqlzx_m8/m12.so) against 16 / 10 (libqlzx.so).
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05km; mkdir -p $O
for r in 1 2; do
  for l in libqlzx.so libqlzx_u12.so libqlzx_u20.so; do
    echo "== c2 $(QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
  done
  for l in libqlzx.so libqlzx_m8.so libqlzx_m12.so; do
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c5_$l.json')); print('== c5 $l', d['value'], d['digest']['xor_output_crc32'])"
  done
done
