#!/bin/bash
# Round 3 K2b bring-up: the byte-parallel K2 stress tests, then the whole GPU suite, then c2
# timing of the new K2 (libqlzx.so) and the item K2 (libqlzx_items.so, -DQLZX_K2_ITEMS).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_bytes.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03_k2b_stress.log 2>&1
rc=$?; tail -15 gpurun_out/r03_k2b_stress.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r03_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for lib in libqlzx.so libqlzx_items.so; do
  QLZX_LIB=gobeansdb_amd/$lib timeout -k 10 180 python -u tools/exp_time.py 1048576 16384 5 2>&1 | grep -v amdgpu.ids || exit 1
done
