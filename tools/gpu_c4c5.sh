#!/bin/bash
# Refresh c4 (.data replay, device-only + pipelined end-to-end + CPU leg) and c5 (400 GiB mixed) at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c4c5
mkdir -p $O
timeout -k 10 700 python3 -u tools/bench_replay.py > $O/c4.json 2> $O/c4.err || { tail $O/c4.err; exit 1; }
cat $O/c4.json
timeout -k 10 600 python3 -u bench.py --config c5 > $O/c5.json 2> $O/c5.err || { tail $O/c5.err; exit 1; }
cat $O/c5.json
