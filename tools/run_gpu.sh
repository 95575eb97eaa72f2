set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r01b
PMC_BENCH_ARGS="--blocks 131072 --steps 1 --warmup 0 --no-cpu" bash tools/pmc.sh r01b/pmc "FETCH_SIZE" "WRITE_SIZE" > gpurun_out/r01b/pmc.txt 2>&1 || { tail gpurun_out/r01b/pmc.txt; exit 1; }
python tools/traffic.py gpurun_out/r01b/pmc 131072 gpurun_out/r01b/traffic.json > /dev/null
timeout -k 10 600 python bench.py --traffic-json gpurun_out/r01b/traffic.json > gpurun_out/r01b/bench.json 2> gpurun_out/r01b/bench.err || { tail gpurun_out/r01b/bench.err; exit 1; }
cat gpurun_out/r01b/bench.json
bash tools/prof.sh r01b/prof --no-cpu --traffic-json gpurun_out/r01b/traffic.json | grep "k_dec" | cut -c1-50,140-260
