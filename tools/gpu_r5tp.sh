#!/bin/bash
# Encoder ticket prefetch A/B (libqlzx_t0.so = without): encoder tests, then the c3 leg and the
# per-class cost interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05tp; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encode_wg.py tests/test_gpu_codec.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for l in libqlzx_t0.so libqlzx.so; do
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu > $O/c3_$l.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c3_$l.json')); print('== c3 $l', d['ms_per_step'])"
  done
done
for l in libqlzx_t0.so libqlzx.so; do
  echo "== $l"; QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 300 python3 tools/enc_prof.py 8192 65536 2>&1 | grep -v amdgpu.ids | head -3
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 300 python3 tools/enc_prof.py 16384 16384 2>&1 | grep -v amdgpu.ids | head -3
done
