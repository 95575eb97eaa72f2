#!/bin/bash
# Scheduler-strategy A/B of the whole library (-mllvm -amdgpu-sched-strategy=...): libqlzx_si.so =
# max-ilp, libqlzx_sm.so = max-memory-clause, libqlzx_sii.so = iterative-ilp, libqlzx.so = default.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05ss; mkdir -p $O
for r in 1 2; do
  for l in libqlzx.so libqlzx_si.so libqlzx_sm.so libqlzx_sii.so; do
    echo "== c2 $(QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 200 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tail -1)"
    QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_c5.py --total-gib 64 > $O/c5_$l.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/c5_$l.json')); print('== c5 $l', d['value'], d['digest']['xor_output_crc32'])"
  done
done
for l in libqlzx.so libqlzx_si.so libqlzx_sm.so libqlzx_sii.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 300 python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu > $O/c3_$l.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_$l.json')); print('== c3 $l', d['ms_per_step'])"
done
