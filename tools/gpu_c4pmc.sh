#!/bin/bash
# c4 replay kernels: FETCH_SIZE / WRITE_SIZE per dispatch (1000 MiB chunk, device-only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c4pmc
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- \
    python3 tools/bench_replay.py --chunk-mib 1000 --files 1 --steps 1 --no-cpu > $O/$c.json 2> $O/$c.err || { tail $O/$c.err; exit 1; }
done
python3 tools/pmc_sum.py $O | grep -A2 "rp_\|dec_"
