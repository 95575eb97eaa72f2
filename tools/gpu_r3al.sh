#!/bin/bash
# Encoder next-block ticket taken one block ahead (tka) vs at the block boundary (notka):
# encoder parity, per-class cost, c3 timing.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03al; mkdir -p $O
QLZX_LIB=gobeansdb_amd/libqlzx_tka.so timeout -k 10 500 python -u -m pytest tests/test_gpu_encode_wg.py tests/test_gpu_sample_parity.py tests/test_gpu_codec.py tests/test_gpu_large.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for t in tka notka; do
  echo "== $t"
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 200 python -u tools/enc_prof.py 16384 65536 2>&1 | grep -v amdgpu.ids | head -4 || exit 1
done
for r in 1 2; do for t in tka notka; do
  echo -n "$t "; QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])" || exit 1
done; done
