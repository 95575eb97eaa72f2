#!/bin/bash
# Round 3: the whole GPU suite, then the driver's default bench line (c2 + crc + c3 + c4 + c5).
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
rc=$?; tail -5 gpurun_out/r03_bench.err; cat gpurun_out/r03_bench.json; exit $rc
