#!/bin/bash
# Parity gate + interleaved A/B timing of decoder builds (round 6).
# usage: TEST_TAG=tag [AB_REPS=2] tools/gpu_ab.sh tag1 tag2 ...  (gobeansdb_amd/libqlzx_TAG.so, "head" = in-tree lib)
# The parity subset runs on $TEST_TAG's library; each tag is then timed by exp_time.py on c2 (1 M x 16 KiB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-ab}; mkdir -p $O
lib() { if [ "$1" = head ]; then echo $PWD/gobeansdb_amd/libqlzx.so; else echo $PWD/gobeansdb_amd/libqlzx_$1.so; fi; }
if [ -n "$TEST_TAG" ]; then
  QLZX_LIB=$(lib $TEST_TAG) timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      ${TESTS:-tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_decode_chunk.py tests/test_gpu_replay.py tests/test_gpu_large.py} \
      > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
: > $O/ab.txt
for r in $(seq ${AB_REPS:-2}); do
  for t in "$@"; do
    QLZX_LIB=$(lib $t) timeout -k 10 180 python -u tools/exp_time.py ${AB_N:-1048576} ${AB_BS:-16384} 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$t /" >> $O/ab.txt || { cat $O/ab.txt; exit 1; }
  done
done
cat $O/ab.txt
