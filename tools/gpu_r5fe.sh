#!/bin/bash
# K2 A/B: far loads of non-jumping bytes issued before the pointer jumping (libqlzx.so) against
# HEAD (libqlzx_f0.so): decode parity tests, then c2 / c5 / c4 interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05fe; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode_chunk.py tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_replay.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for l in libqlzx_f0.so libqlzx.so; do
    echo "== c2 $(QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
    echo "== c2crc $(QLZX_CRC=1 QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c5_$l.json')); print('== c5 $l', d['value'])"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 2 --no-cpu > $O/c4_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c4_$l.json')); print('== c4 $l', d['value'])"
  done
done
