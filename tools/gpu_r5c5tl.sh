set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05c5tl; mkdir -p $O
for l in libqlzx_p4.so libqlzx.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$l -o kt -- python3 tools/bench_c5.py --total-gib 16 > $O/c5_$l.json 2>/dev/null || exit 1
  f=$(find $O/kt_$l -name "*kernel_trace.csv" | head -1); cp $f $O/trace_$l.csv; rm -rf $O/kt_$l
  echo "== $l"; python3 tools/call_timeline.py $O/trace_$l.csv k_order_count -1 | tee $O/tl_$l.txt
done
