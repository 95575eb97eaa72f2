#!/bin/bash
# c3 encoder HBM traffic: FETCH_SIZE / WRITE_SIZE passes over 65536 x 64 KiB image-like blocks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c3pmc
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- \
      python3 bench.py --config c3 --blocks 65536 --steps 1 --warmup 0 --no-cpu > $O/pmc_$c.json 2> $O/pmc_$c.err || { tail $O/pmc_$c.err; exit 1; }
done
python3 tools/traffic.py $O 65536 $O/c3_traffic.json k_encode_wg && cat $O/c3_traffic.json
