#!/bin/bash
# Round 4 end: the full -m gpu suite, smoke(), and the default bench line under a kernel trace
# (c2 + c3 + c4 replay + c5 legs), rocprof stats kept for profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04final}; mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
      > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
    python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
python3 tools/kstats.py $(find $O/trace -name "*kernel_trace.csv" | head -1) > $O/kernels.txt
head -20 $O/kernels.txt
