#!/bin/bash
# Build experiment variants of libqlzx.so: tools/build_variants.sh TAG "-DFLAG ..." [TAG "-D..."]...
# -> gobeansdb_amd/libqlzx_TAG.so (git-ignored; travels to the GPU box with gpurun).  Built as
# gobeansdb_amd/build.py builds the release library: qlzx_api.hip with QLZX_SPLIT_K1/K2, and K1 +
# K2 without CRC in qlzx_k2.hip under the iterative-ilp scheduler, then linked; TAG flags go to both
# units (a flag containing -amdgpu-sched-strategy for qlzx_k2.hip overrides the default one).
cd "$(dirname "$0")/.."
B="hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC --offload-compress -Wno-unused-function -Wno-unused-parameter -I include"
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2
  o=gobeansdb_amd/libqlzx_$tag
  k2sched="-mllvm -amdgpu-sched-strategy=iterative-ilp"
  case "$flags" in *amdgpu-sched-strategy*) k2sched="";; esac
  ( $B -c -DQLZX_SPLIT_K1=1 $flags -DQLZX_SPLIT_K2=1 -o $o.api.o gobeansdb_amd/csrc/qlzx_api.hip &&
    $B -c -DQLZX_SPLIT_K1=1 $flags $k2sched -o $o.k2.o gobeansdb_amd/csrc/qlzx_k2.hip &&
    hipcc --offload-arch=gfx950 -fPIC -shared -o $o.so $o.api.o $o.k2.o; rm -f $o.api.o $o.k2.o ) &
done
wait
