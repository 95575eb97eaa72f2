#!/bin/bash
# iterative-ilp scheduler (libqlzx_sii.so) against the default (libqlzx.so): the GPU test suite on
# the variant, then c2 CRC / c3 / c4 / single-call latency interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05ss2; mkdir -p $O
QLZX_LIB=$PWD/gobeansdb_amd/libqlzx_sii.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for l in libqlzx.so libqlzx_sii.so; do
    echo "== c2crc $(QLZX_CRC=1 QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 300 python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu > $O/c3_$l.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/c3_$l.json')); print('== c3 $l', d['ms_per_step'])"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 2 --no-cpu > $O/c4_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c4_$l.json')); print('== c4 $l', d['value'])"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 300 python -u tools/bench_single.py --calls 1000 --values 1024 --threads 0 --out $O/single_$l.json > /dev/null 2>&1 || exit 1
    python3 -c "
import json; d=json.load(open('$O/single_$l.json'))
print('== single $l', [(r['bytes'], r['gpu_decompress_us'], r['gpu_compress_us'], r['gpu_crc32_us']) for r in d['rows']])"
  done
done
