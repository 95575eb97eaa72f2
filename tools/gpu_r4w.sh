#!/bin/bash
# Round 4: A/B of single-call builds: solo tests, then 1/16-thread qlz_decompress aggregate and the
# per-call latency table of each library (paths relative to the repo root).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04w}; mkdir -p $O
gcc -O2 -pthread -o $O/mt_single tools/mt_single.c -ldl || exit 1
python3 - $O <<'PY' || exit 1
import sys; sys.path.insert(0, '.')
from oracle import oracle as O
for n in (4096, 16384, 65536):
    open(f'{sys.argv[1]}/c{n}.bin', 'wb').write(O.compress(O.gen_text(0x5EED2026, n, n)))
PY
for l in "$@"; do
  echo "== $l" | tee -a $O/ab.txt
  QLZX_LIB=$PWD/$l timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solo.py \
      > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log | tee -a $O/ab.txt
  for n in 4096 16384; do
    for t in 1 16; do
      timeout -k 10 60 $O/mt_single $PWD/$l $O/c$n.bin $t 2 | tee -a $O/ab.txt || exit 1
    done
  done
done
