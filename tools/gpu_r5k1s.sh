#!/bin/bash
# K1 (k_dec_parse6) moved into qlzx_k2.hip's unit as well (libqlzx_k1s.so, -DQLZX_SPLIT_K1=1) against
# gobeansdb_amd/build.py) against the one-unit build (libqlzx_k1s.so): the GPU suite on the split
# (interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05k1s; mkdir -p $O
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_k1s.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
for r in 1 2; do
  for l in libqlzx_k1s.so libqlzx.so; do
    echo "== c2 $(QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
    echo "== c2crc $(QLZX_CRC=1 QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c5_$l.json')); print('== c5 $l', d['value'], d['digest']['xor_output_crc32'])"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 2 --no-cpu > $O/c4_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c4_$l.json')); print('== c4 $l', d['value'])"
  done
done
