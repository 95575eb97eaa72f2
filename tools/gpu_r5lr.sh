#!/bin/bash
# Round 5: A/B of K1 with per-lane rings (libqlzx_lr.so, -DQLZX_K1_LANE_RING) against HEAD --
# parity tests on the variant, then interleaved c2 timings and a c5 slice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05lr}; mkdir -p $O
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_lr.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_decode_chunk.py tests/test_gpu_replay.py tests/test_gpu_large.py \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for l in libqlzx.so libqlzx_lr.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 120 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt || exit 1
done; done
for l in libqlzx.so libqlzx_lr.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
  python3 -c "import json; r=json.load(open('$O/c5_$l.json')); print('$l c5', r['value'])" | tee -a $O/ab.txt
done
