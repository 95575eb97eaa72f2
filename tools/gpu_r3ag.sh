#!/bin/bash
# Encoder best-match candidate reads: candidates staged in LDS (candlds), LDS reads only for
# candidates that can match (okread), both, vs HEAD (ehead): parity of each, c3 timing, per-class.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ag; mkdir -p $O
for t in candlds okread both; do
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 300 python -u -m pytest tests/test_gpu_encode_wg.py tests/test_gpu_sample_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests_$t.log 2>&1 || { tail -30 $O/tests_$t.log; exit 1; }
  echo "$t: $(tail -1 $O/tests_$t.log)"
done
for t in candlds okread both ehead; do
  echo "== $t"
  QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 200 python -u tools/enc_prof.py 16384 65536 2>&1 | grep -v amdgpu.ids | head -4 || exit 1
done
for r in 1 2; do for t in candlds okread both ehead; do
  echo -n "$t "; QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'])" || exit 1
done; done
