#!/bin/bash
# c3 compress bench: a short run at 64 K blocks, then the full 1 M x 64 KiB config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --mode compress --block-size 65536 --blocks 65536 --steps 3 --warmup 1 \
    --cpu-seconds 5 > gpurun_out/c3_small.json 2> gpurun_out/c3_small.err || { tail -20 gpurun_out/c3_small.err; exit 1; }
cat gpurun_out/c3_small.json; tail -4 gpurun_out/c3_small.err
timeout -k 10 500 python -u bench.py --mode compress --block-size 65536 --steps 5 --warmup 1 \
    --cpu-seconds 15 > gpurun_out/c3_full.json 2> gpurun_out/c3_full.err || { tail -20 gpurun_out/c3_full.err; exit 1; }
cat gpurun_out/c3_full.json; tail -4 gpurun_out/c3_full.err
