#!/bin/bash
# Round 3 quick loop: K2 stress + decode parity tests, then interleaved c2 timing of the
# variants named on the command line (gobeansdb_amd/libqlzx_TAG.so), then the phase profile.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_bytes.py tests/test_gpu_codec.py tests/test_gpu_sample_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_quick_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh "$@" || exit 1
QLZX_LIB=gobeansdb_amd/libqlzx_prof.so timeout -k 10 120 python -u tools/phase_prof.py 131072 16384 2>&1 | grep -v amdgpu.ids
