#!/bin/bash
# K2 without CRC in its own translation unit with the iterative-ilp scheduler (in-tree libqlzx.so,
# gobeansdb_amd/build.py) against the one-unit build (libqlzx_ns.so): the GPU suite on the split
# build, smoke, then c2 / c2+CRC / c5 / c4 interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05sp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
for r in 1 2; do
  for l in libqlzx_ns.so libqlzx.so; do
    echo "== c2 $(QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
    echo "== c2crc $(QLZX_CRC=1 QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c5_$l.json')); print('== c5 $l', d['value'], d['digest']['xor_output_crc32'])"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 2 --no-cpu > $O/c4_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c4_$l.json')); print('== c4 $l', d['value'])"
  done
done
