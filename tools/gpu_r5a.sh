#!/bin/bash
# Round 5: v5 decoder pair -- decode parity tests, then c2 A/B against the round-4 pair.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05a}; mkdir -p $O
QLZX_LIB=$PWD/${TEST_LIB:-gobeansdb_amd/libqlzx.so} timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_codec.py tests/test_gpu_sample_parity.py ${EXTRA_TESTS} 2>&1 | tail -30 | tee $O/tests.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
: > $O/ab.txt
for rep in 1 2; do
  for l in ${VARIANTS:-v4 v5}; do
    lib=gobeansdb_amd/libqlzx_$l.so; [ $l = head ] && lib=gobeansdb_amd/libqlzx.so
    QLZX_LIB=$PWD/$lib timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt
    [ ${PIPESTATUS[0]} -ne 0 ] && exit 1
  done
done
exit 0
