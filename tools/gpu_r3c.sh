#!/bin/bash
# CRC tests, A/B of the record CRC in a separate kernel (sep) vs inside K1 (k1crc), K2b phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
O=gpurun_out/r03c
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_sample_parity.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
AB_CRC=1 bash tools/gpu_ab.sh sep k1crc || exit 1
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids
