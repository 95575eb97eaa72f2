#!/bin/bash
# Ring-tile encoder: parity tests of the encoder, then per-class cost and the c3 leg.
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05rt; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_encode_wg.py tests/test_gpu_codec.py > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/enc_prof.py 8192 65536 > $O/enc_prof.txt 2>&1 || exit 1
cat $O/enc_prof.txt
timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
cat $O/c3.json
