#!/bin/bash
# Round 4: c3 encoder evidence at HEAD -- FETCH/WRITE traffic of the 64 KiB encoder, cost per input
# class and per-phase cycles (profile build), kernel trace of a c3 run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04z}; mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- \
      python3 bench.py --config c3 --blocks 65536 --steps 1 --warmup 0 --no-cpu > $O/pmc_$c.json 2> $O/pmc_$c.err || { tail $O/pmc_$c.err; exit 1; }
done
python3 tools/traffic.py $O 65536 $O/r04_c3_traffic.json k_encode_wg > /dev/null && cat $O/r04_c3_traffic.json || exit 1
timeout -k 10 300 python -u tools/enc_prof.py 8192 65536 2>&1 | grep -v amdgpu.ids | tee $O/enc_prof.txt || exit 1
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 300 python -u tools/enc_phase.py 8192 65536 2>&1 | grep -v amdgpu.ids | tee $O/enc_phase.txt || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c3 -- \
    python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
cat $O/c3.json
