#!/bin/bash
# Single-call compress: the widest encoder workgroup for a lone block (cap64 / cap16) vs the one its
# size selects (cap4): single-call tests, then the per-call latency table for each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03s; mkdir -p $O
QLZX_LIB=gobeansdb_amd/libqlzx_cap64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_solo.py tests/test_gpu_level1.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in cap4 cap16 cap64; do
  echo "== $t"
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 300 python -u tools/bench_single.py --calls 300 --out $O/single_$t.json > $O/single_$t.log 2>&1 || { tail -20 $O/single_$t.log; exit 1; }
  cat $O/single_$t.log | grep bytes
done
