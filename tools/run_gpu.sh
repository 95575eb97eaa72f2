set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/r14_pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/r14_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/bench_replay.py --files 13 > gpurun_out/c4_r14.json 2> gpurun_out/c4_r14.err; rc=$?; tail -2 gpurun_out/c4_r14.err; cat gpurun_out/c4_r14.json; exit $rc
