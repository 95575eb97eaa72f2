#!/bin/bash
# Round 4: single-call request path (qlzx_service.hip) -- single-call tests, latency table, the
# 16-thread aggregate qlz_decompress rate (tools/mt_single.c) against the reference, and a kernel
# trace of the latency run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04c}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_codec.py tests/test_gpu_solo.py \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
gcc -O2 -pthread -o $O/mt_single tools/mt_single.c -ldl || exit 1
python3 - <<'PY' || exit 1
import sys; sys.path.insert(0, '.')
from oracle import oracle as O
for n in (4096, 16384, 65536):
    open(f'gpurun_out/{sys.argv[1] if len(sys.argv) > 1 else "r04c"}/c{n}.bin', 'wb').write(O.compress(O.gen_text(0x5EED2026, n, n)))
PY
for n in 4096 16384 65536; do
  for t in 1 16; do
    timeout -k 10 60 $O/mt_single $PWD/gobeansdb_amd/libqlzx.so $O/c$n.bin $t 2 | tee -a $O/mt.jsonl || exit 1
    timeout -k 10 60 $O/mt_single $PWD/oracle/_ref/libqlzref.so $O/c$n.bin $t 2 | tee -a $O/mt.jsonl || exit 1
  done
done
timeout -k 10 300 python -u tools/bench_single.py --calls 1000 --threads 0 --out $O/single_call.json 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- \
    python3 tools/bench_single.py --calls 200 --threads 0 > $O/trace.txt 2>&1 || { tail $O/trace.txt; exit 1; }
python3 tools/kstats.py $(find $O/trace -name "*kernel_trace.csv" | head -1) | tee $O/kernels.txt
