#!/bin/bash
# Round 5: K1 variants on the full workloads -- p4 (round-4 k_dec_parse4), k2set (per-lane ring,
# loads stored one iteration later), k3set (two iterations later): parity on k3set, c2, full c5,
# c4 4 x 4000 MiB.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05k3}; mkdir -p $O
LIBS=${LIBS:-"p4 k2set k3set"}
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_${TEST_TAG:-k3set}.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_decode_chunk.py tests/test_gpu_replay.py tests/test_gpu_large.py \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for l in $LIBS; do
  QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_$l.so timeout -k 10 120 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | sed "s/^/$l /" | tee -a $O/ab.txt || exit 1
  QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_$l.so timeout -k 10 300 python3 tools/bench_c5.py > $O/c5_$l.json 2>/dev/null || exit 1
  QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_$l.so timeout -k 10 300 python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 2 --no-cpu --pin-records 16 > $O/c4_$l.json 2>/dev/null || exit 1
  python3 -c "import json; r=json.load(open('$O/c5_$l.json')); q=json.load(open('$O/c4_$l.json')); print('$l c5', r['value'], 'c4', q['value'])" | tee -a $O/ab.txt
done
