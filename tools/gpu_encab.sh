#!/bin/bash
# A/B of encoder builds: c3 (1 M x 64 KiB image-like, fused CRC) ms per step for each library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for l in "$@"; do
  if [ "$l" = default ]; then lib=$PWD/gobeansdb_amd/libqlzx.so; else lib=$PWD/$l; fi
  QLZX_LIB=$lib timeout -k 10 400 python -u bench.py --config c3 --no-cpu --steps 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l', d['ms_per_step'], 'ms', d['value'], 'GiB/s')" || exit 1
done
