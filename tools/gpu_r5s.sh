#!/bin/bash
# Round 5: single-call evidence over >= 1024 DISTINCT values per size, both sides -- service tests,
# the small-block decoder's phase stamps, the latency table (tools/bench_single.py) and the 1/16
# pthread aggregate qlz_decompress rate (tools/mt_single.c) of this library and the reference.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05s}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_service.py tests/test_gpu_solo.py \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/solo_prof.py 300 2>&1 | grep -v amdgpu.ids | tee $O/solo_prof.txt || exit 1
timeout -k 10 400 python -u tools/bench_single.py --calls 1000 --values 1024 --threads 16 --dump $O --out $O/single_call.json 2>&1 | grep -v amdgpu.ids || exit 1
gcc -O2 -pthread -o $O/mt_single tools/mt_single.c -ldl || exit 1
for n in 4096 16384 65536; do
  for t in 1 16; do
    timeout -k 10 60 $O/mt_single $PWD/gobeansdb_amd/libqlzx.so $O/values_$n.bin $t 2 | tee -a $O/mt.jsonl || exit 1
    timeout -k 10 60 $O/mt_single $PWD/oracle/_ref/libqlzref.so $O/values_$n.bin $t 2 | tee -a $O/mt.jsonl || exit 1
  done
done
rm -f $O/values_*.bin
