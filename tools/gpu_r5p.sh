#!/bin/bash
# Round 5: c4 replay work -- parity tests, c2 timing (unchanged path check), then a kernel trace
# of tools/bench_replay.py (two 4000 MiB chunk files) with the per-call kernel timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05p}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_replay.py \
    tests/test_gpu_codec.py tests/test_gpu_sample_parity.py tests/test_gpu_decode_chunk.py tests/test_gpu_large.py \
    > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tee $O/c2.txt || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
    python3 tools/bench_replay.py --chunk-mib 4000 --files 4 --steps 3 --no-cpu --pin-records 64 \
    > $O/out.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
f=$(find $O/kt -name "*kernel_trace.csv" | head -1); cp $f $O/trace.csv; rm -rf $O/kt
python3 tools/call_timeline.py $O/trace.csv k_rp_scan 8 | tee $O/timeline.txt
python3 -c "import json,sys; r=json.load(open('$O/out.json')); print('c4', r['value'], r['ms_per_step'], r['end_to_end_pipelined']['gib_per_s_chunk'], r['digest']['xor_value_crc32'])"
