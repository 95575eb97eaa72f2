#!/bin/bash
# Small-block decoder step 1b A/B: parity tests, phase stamps (libqlzx_prof.so vs libqlzx_pc0.so),
# then single-call latency and the 16-pthread aggregate, variant (libqlzx.so) against HEAD
# (libqlzx_c0.so).  Round 5: interleaved chains, static candidates, then token pairs.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05sc; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solo.py tests/test_gpu_service.py tests/test_gpu_codec.py \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for l in libqlzx_pc0.so libqlzx_prof.so; do
  echo "== $l"; QLZX_LIB=gobeansdb_amd/$l timeout -k 10 120 python -u tools/solo_prof.py 300 2>&1 | grep -v amdgpu.ids | tee $O/solo_prof_$l.txt || exit 1
done
timeout -k 10 200 python -u tools/bench_single.py --calls 1000 --values 1024 --threads 0 --dump $O --out $O/single_dump.json > /dev/null 2>&1 || exit 1
gcc -O2 -pthread -o $O/mt_single tools/mt_single.c -ldl || exit 1
for l in libqlzx_c0.so libqlzx.so libqlzx_c0.so libqlzx.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 300 python -u tools/bench_single.py --calls 1000 --values 1024 --threads 0 --out $O/single_$l.json 2>&1 | grep -v amdgpu.ids > $O/single_$l.txt || exit 1
  python3 -c "
import json; d=json.load(open('$O/single_$l.json'))
rows=d.get('rows') or d.get('latency',{}).get('rows')
print('== $l', [(r['bytes'], r['gpu_decompress_us']) for r in rows])"
  for n in 4096 16384; do timeout -k 10 60 $O/mt_single $PWD/gobeansdb_amd/$l $O/values_$n.bin 16 2 || exit 1; done
done
rm -f $O/values_*.bin
