#!/bin/bash
# Tiled pass B of the encoder's sort: encoder parity tests, phase stamps against the untiled pass
# (libqlzx_prof0.so), then the c3 leg with and without it (libqlzx_t0.so).
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05tb; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encode_wg.py tests/test_gpu_codec.py tests/test_gpu_large.py > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for l in libqlzx_prof0.so libqlzx_prof.so; do
  echo "== $l"
  KINDS=noisy,text QLZX_LIB=gobeansdb_amd/$l timeout -k 10 300 python -u tools/enc_phase.py 4096 65536 2>&1 | grep -v amdgpu.ids | tee $O/phase_$l.txt || exit 1
done
for l in libqlzx_t0.so libqlzx.so libqlzx_t0.so libqlzx.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu > $O/c3_$l.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c3_$l.json')); print('$l', d['ms_per_step'], d['value'])"
done
