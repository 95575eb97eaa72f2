#!/bin/bash
# Interleaved c2 timing of library variants on one box: tools/gpu_ab.sh TAG1 TAG2 ...
# (gobeansdb_amd/libqlzx_TAG.so; each run checks its round trip first).  AB_CRC=1 adds a
# pass with the fused record-CRC verify per variant.
for r in 1 2; do
  for t in "$@"; do
    QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
    if [ -n "$AB_CRC" ]; then
      QLZX_CRC=1 QLZX_LIB=gobeansdb_amd/libqlzx_$t.so timeout -k 10 120 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
    fi
  done
done
