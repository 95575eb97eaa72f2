set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -x -q -m gpu > gpurun_out/r9_pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r9_pytest.txt; exit 1; }
tail -2 gpurun_out/r9_pytest.txt
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 200 python tools/phase_prof.py > gpurun_out/ph8.txt 2>&1 && cat gpurun_out/ph8.txt
bash tools/prof.sh p8 --blocks 262144 --steps 3 --warmup 1 --cpu-seconds 0 | grep "k_dec"
