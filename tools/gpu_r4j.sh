#!/bin/bash
# Round 4: single-call path with the small-block LDS decoder -- solo/codec tests, phase stamps,
# latency table and the 16-thread aggregate against the reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04j}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solo.py tests/test_gpu_codec.py \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/solo_prof.py 300 2>&1 | grep -v amdgpu.ids | tee $O/solo_prof.txt || exit 1
gcc -O2 -pthread -o $O/mt_single tools/mt_single.c -ldl || exit 1
python3 - $OUT <<'PY' || exit 1
import sys; sys.path.insert(0, '.')
from oracle import oracle as O
for n in (4096, 16384, 65536):
    open(f'gpurun_out/{sys.argv[1] if len(sys.argv) > 1 else "r04j"}/c{n}.bin', 'wb').write(O.compress(O.gen_text(0x5EED2026, n, n)))
PY
for n in 4096 16384 65536; do
  for t in 1 16; do
    timeout -k 10 60 $O/mt_single $PWD/gobeansdb_amd/libqlzx.so $O/c$n.bin $t 2 | tee -a $O/mt.jsonl || exit 1
  done
done
timeout -k 10 300 python -u tools/bench_single.py --calls 1000 --threads 0 --out $O/single_call.json 2>&1 | grep -v amdgpu.ids || exit 1
