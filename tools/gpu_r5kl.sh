#!/bin/bash
# K1 step budget for the later chunks of mixed calls (A/B): libqlzx_l3.so = 16 from chunk 3,
# libqlzx_l2.so = 16 from chunk 2, libqlzx_l3s.so = 7 from chunk 3, libqlzx.so = 10 throughout.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05kl; mkdir -p $O
for r in 1 2; do
  for l in libqlzx.so libqlzx_l3.so libqlzx_l2.so libqlzx_l3s.so; do
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c5_$l.json')); print('== c5 $l', d['value'], d['digest']['xor_output_crc32'])"
  done
done
