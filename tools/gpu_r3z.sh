#!/bin/bash
# Encoder evidence at HEAD: per-phase cycles (profile build), c3 rocprof kernel trace, c3 PMC
# traffic (FETCH_SIZE, WRITE_SIZE passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03z; mkdir -p $O
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 200 python -u tools/enc_phase.py 4096 65536 2>&1 | grep -v amdgpu.ids | tee $O/enc_phase.txt || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o run -- \
    python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu > $O/c3prof_bench.json 2> $O/c3prof.err || { tail $O/c3prof.err; exit 1; }
head -c 300 $O/c3prof_bench.json; echo
python3 tools/kstats.py $(find $O/c3prof -name "*kernel_trace.csv" | head -1) encode crc | tee $O/c3_medians.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/c3pmc_$c -o run -- \
      python3 bench.py --config c3 --blocks 65536 --steps 1 --warmup 0 --no-cpu > $O/c3pmc_$c.json 2> $O/c3pmc_$c.err || { tail $O/c3pmc_$c.err; exit 1; }
done
python3 tools/traffic.py $O 65536 $O/r03_c3_traffic.json k_encode_wg && cat $O/r03_c3_traffic.json
