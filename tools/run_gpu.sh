set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/c4prof2
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/r11_pytest.txt 2>&1; rc=$?
tail -15 gpurun_out/r11_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof2 -o run -- python3 tools/bench_replay.py --files 4 --steps 2 > gpurun_out/c4prof2/out.json 2> gpurun_out/c4prof2/err.txt; rc=$?
tail -2 gpurun_out/c4prof2/err.txt; cat gpurun_out/c4prof2/out.json; cut -c1-150 gpurun_out/c4prof2/run_kernel_stats.csv | grep -v "at::\|rocprim" | head -16; exit $rc
