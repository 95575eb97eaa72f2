#!/bin/bash
# Round-2 check: box CPU facts, GPU tests, single-call latency, c2 bench with the CPU leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r2a
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > gpurun_out/r2a/cpu.txt 2>&1
cat gpurun_out/r2a/cpu.txt
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations=8 > gpurun_out/r2a/pytest.txt 2>&1
rc=$?; tail -14 gpurun_out/r2a/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_single.py --calls 200 --out gpurun_out/r2a/single.json > gpurun_out/r2a/single.txt 2>&1 || { tail gpurun_out/r2a/single.txt; exit 1; }
cat gpurun_out/r2a/single.txt
timeout -k 10 400 python -u bench.py --cpu-seconds 10 > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err || { tail -20 gpurun_out/r2a/bench.err; exit 1; }
cat gpurun_out/r2a/bench.json
