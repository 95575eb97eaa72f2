#!/bin/bash
# Experiment: lane-per-block decoder (QLZX_DECODE=lane8) vs the K1/K2 path on c2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/l8
QLZX_DECODE=lane8 timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/l8/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/l8/pytest.txt; [ $rc -le 1 ] || exit $rc
QLZX_DECODE=lane8 timeout -k 10 400 python bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/l8/bench_lane8.json 2> gpurun_out/l8/bench_lane8.err || { tail gpurun_out/l8/bench_lane8.err; exit 1; }
cat gpurun_out/l8/bench_lane8.json
timeout -k 10 400 python bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/l8/bench_wave.json 2> gpurun_out/l8/bench_wave.err || { tail gpurun_out/l8/bench_wave.err; exit 1; }
cat gpurun_out/l8/bench_wave.json
