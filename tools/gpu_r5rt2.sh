#!/bin/bash
# Encoder phase stamps: ring tiles (libqlzx_prof.so) against the global sort (libqlzx_prof0.so).
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
O=gpurun_out/r05rt2; mkdir -p $O
for l in libqlzx_prof0.so libqlzx_prof.so; do
  echo "== $l"
  KINDS=noisy,text,random QLZX_LIB=gobeansdb_amd/$l timeout -k 10 300 python -u tools/enc_phase.py 4096 65536 2>&1 | grep -v amdgpu.ids | tee $O/phase_$l.txt || exit 1
done
