set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r01
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/r01/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r01/pytest.txt; exit 1; }
tail -2 gpurun_out/r01/pytest.txt
PMC_BENCH_ARGS="--blocks 131072 --steps 1 --warmup 0 --no-cpu" bash tools/pmc.sh r01/pmc "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/r01/pmc.txt 2>&1 || { echo "pmc failed"; tail gpurun_out/r01/pmc.txt; exit 1; }
python tools/traffic.py gpurun_out/r01/pmc 131072 gpurun_out/r01/traffic.json
timeout -k 10 600 python bench.py --traffic-json gpurun_out/r01/traffic.json > gpurun_out/r01/bench.json 2> gpurun_out/r01/bench.err || { echo "bench failed"; tail gpurun_out/r01/bench.err; exit 1; }
cat gpurun_out/r01/bench.json
bash tools/prof.sh r01/prof --no-cpu --traffic-json gpurun_out/r01/traffic.json | grep -v "at::\|__amd"
