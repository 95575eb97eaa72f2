#!/bin/bash
# Round 5: K1 rounds per iteration (2 vs 3) and step budgets: parity on one variant, interleaved
# c2, then c5 / c4 slices.  LIBS: variant tags (libqlzx_TAG.so); head = libqlzx.so.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05m3}; mkdir -p $O
LIBS=${LIBS:-"head m3 m3k14 m3k20"}
lib() { [ $1 = head ] && echo gobeansdb_amd/libqlzx.so || echo gobeansdb_amd/libqlzx_$1.so; }
QLZX_LIB=$PWD/$(lib ${TEST_TAG:-m3}) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_decode_chunk.py tests/test_gpu_replay.py \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for l in $LIBS; do
  QLZX_LIB=$PWD/$(lib $l) timeout -k 10 120 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$l /" | tee -a $O/ab.txt || exit 1
done; done
for l in $LIBS; do
  QLZX_LIB=$PWD/$(lib $l) timeout -k 10 200 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
  QLZX_LIB=$PWD/$(lib $l) timeout -k 10 300 python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 2 --no-cpu --pin-records 16 > $O/c4_$l.json 2>/dev/null || exit 1
  python3 -c "import json; r=json.load(open('$O/c5_$l.json')); q=json.load(open('$O/c4_$l.json')); print('$l c5', r['value'], 'c4', q['value'])" | tee -a $O/ab.txt
done
