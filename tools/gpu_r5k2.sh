#!/bin/bash
# K2 micro A/B: far reads in one divergent region (FAR1) and the unconditional pending flush
# (PEND1).  libqlzx_k0.so = neither, libqlzx_kf.so = FAR1, libqlzx.so = both.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05k2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_decode_chunk.py tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_replay.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for l in libqlzx_k0.so libqlzx_kf.so libqlzx.so; do
    echo "== c2 $l $(QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
  done
done
for l in libqlzx_k0.so libqlzx.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/c5_$l.json')); print('c5 $l', d['value'])"
done
