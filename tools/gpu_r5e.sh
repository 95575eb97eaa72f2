#!/bin/bash
# A/B of early-K1 variants (QLZX_EARLY_K1 = 0, 1 (libqlzx.so), 2, 3) on the c5 leg, then the
# 6-chunk-round timeline of the default and of the best variant.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
for l in libqlzx_e0.so libqlzx.so libqlzx_e2.so libqlzx_e3.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 240 python3 tools/bench_c5.py > $O/c5_$l.json 2>$O/c5_$l.err || exit 1
  echo "== $l $(cat $O/c5_$l.json)"
done
for l in libqlzx.so libqlzx_e2.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$l -o kt -- python3 tools/bench_c5.py --total-gib 16 --round-gib 17 > $O/c5tl_$l.json 2>/dev/null || exit 1
  f=$(find $O/kt_$l -name "*kernel_trace.csv" | head -1); cp $f $O/trace_$l.csv; rm -rf $O/kt_$l
  echo "== $l"; python3 tools/call_timeline.py $O/trace_$l.csv k_order_count -1 | tee $O/tl_$l.txt
done
