set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/r10_pytest.txt 2>&1; rc=$?
tail -30 gpurun_out/r10_pytest.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PMC_BENCH_ARGS="--blocks 131072 --unique 16384 --steps 1 --warmup 0 --no-cpu" bash tools/pmc.sh pmc2 "TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_STALL_MULTI_MISS TCP_UTCL1_THRASHING_STALL" "TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_sum TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TCC_HIT_sum TCC_MISS_sum" 2>&1 | tail -40
