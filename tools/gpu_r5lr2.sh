#!/bin/bash
# Round 5: K1 per-lane-ring step budget sweep (c2 timing + kernel trace of K1/K2 per variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r05lr2}; mkdir -p $O
for l in libqlzx.so libqlzx_lr.so libqlzx_lr10.so libqlzx_lr16.so libqlzx_lr24.so; do
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -k 10 120 python3 tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.txt || exit 1
  QLZX_LIB=$PWD/gobeansdb_amd/$l timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$l -o kt -- \
      python3 tools/exp_time.py 262144 16384 2 > /dev/null 2>&1 || { echo "trace $l failed"; exit 1; }
  python3 tools/kstats.py $(find $O/kt_$l -name "*kernel_trace.csv" | head -1) | grep "dec_" | sed "s/^/$l /" | tee -a $O/ab.txt
  rm -rf $O/kt_$l
done
