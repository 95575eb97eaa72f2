#!/bin/bash
# Build experiment variants of libqlzx.so: tools/build_variants.sh TAG "-DFLAG ..." [TAG "-D..."]...
# -> gobeansdb_amd/libqlzx_TAG.so (git-ignored; travels to the GPU box with gpurun).
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  tag=$1; flags=$2; shift 2
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared --offload-compress -Wno-unused-function -Wno-unused-parameter $flags \
      -I include -o gobeansdb_amd/libqlzx_$tag.so gobeansdb_amd/csrc/qlzx_api.hip &
done
wait
