set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -x -q -m gpu 2>&1 | tail -3 || exit 1
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 200 python tools/phase_prof.py 2>&1 | grep K1
bash tools/prof.sh k1m --blocks 262144 --unique 16384 --steps 3 --warmup 1 --no-cpu | grep "k_dec" | cut -c1-40,150-260 || exit 1
