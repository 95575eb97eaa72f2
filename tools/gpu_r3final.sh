#!/bin/bash
# Round 3 final evidence: full GPU suite, the driver's default bench line, c2 rocprof with and
# without the record CRC, K1/K2 phase stamps, c3 rocprof + PMC traffic + encoder phases,
# single-call latencies.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03final; mkdir -p $O
OUT=r03final bash tools/gpu_r3m.sh || exit 1
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 200 python -u tools/enc_phase.py 4096 65536 2>&1 | grep -v amdgpu.ids > $O/enc_phase.txt || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o run -- \
    python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu > $O/c3prof_bench.json 2> $O/c3prof.err || { tail $O/c3prof.err; exit 1; }
python3 tools/kstats.py $(find $O/c3prof -name "*kernel_trace.csv" | head -1) encode crc | tee $O/c3_medians.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/c3pmc_$c -o run -- \
      python3 bench.py --config c3 --blocks 65536 --steps 1 --warmup 0 --no-cpu > $O/c3pmc_$c.json 2> $O/c3pmc_$c.err || { tail $O/c3pmc_$c.err; exit 1; }
done
python3 tools/traffic.py $O 65536 $O/r03_c3_traffic.json k_encode_wg && cat $O/r03_c3_traffic.json
timeout -k 10 300 python -u tools/bench_single.py --calls 300 --out $O/r03_single_call.json > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -12 $O/single.log
echo done
