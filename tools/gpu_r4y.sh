#!/bin/bash
# Round 4: encoder A/B -- parity (test_gpu_encode_wg + sample parity) and cost per input class for
# each library given (paths relative to the repo root; "default" = the in-tree lib).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04y}; mkdir -p $O
: > $O/ab.txt
for l in "$@"; do
  if [ "$l" = default ]; then lib=$PWD/gobeansdb_amd/libqlzx.so; else lib=$PWD/$l; fi
  echo "== $l" >> $O/ab.txt
  if [ -z "$NOPAR" ]; then
    QLZX_LIB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
        tests/test_gpu_encode_wg.py tests/test_gpu_sample_parity.py -k "encoder or compress" >> $O/ab.txt 2>&1 || { tail -30 $O/ab.txt; exit 1; }
  fi
  QLZX_LIB=$lib timeout -k 10 300 python -u tools/enc_prof.py ${EN:-8192} 65536 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail $O/ab.txt; exit 1; }
done
grep -v "^\.\|passed\|^$" $O/ab.txt
