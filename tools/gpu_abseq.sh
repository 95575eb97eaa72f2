#!/bin/bash
# A/B timing of QLZX_K2=seq experiment builds on 1 M x 16 KiB text (timing only; experiment
# builds may produce wrong bytes: QLZX_EXPERIMENT=1 skips their round-trip gate).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for l in "$@"; do
  if [ "$l" = default ]; then lib=$PWD/gobeansdb_amd/libqlzx.so; else lib=$PWD/$l; fi
  QLZX_K2=${AB_K2:-seq} QLZX_EXPERIMENT=1 QLZX_LIB=$lib timeout -k 10 180 python -u tools/exp_time.py ${AB_N:-1048576} ${AB_BS:-16384} 5 2>&1 | grep -v amdgpu.ids || exit 1
done
