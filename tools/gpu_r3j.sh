#!/bin/bash
# Encoder: candidates staged in LDS (candlds) vs global loads (main): parity, per-class cost, c3.
# K2b: HEAD (separate pointer array) vs main (pointer array aliasing the marker ring), c2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03j; mkdir -p $O
QLZX_LIB=gobeansdb_amd/libqlzx_candlds.so timeout -k 10 400 python -u -m pytest tests/test_gpu_encode_wg.py tests/test_gpu_sample_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for t in candlds main; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 200 python -u tools/enc_prof.py 16384 65536 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
done
for r in 1 2; do for t in candlds main; do
  echo "== $t"; QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])" || exit 1
done; done
for r in 1 2; do for t in head main; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done; done
