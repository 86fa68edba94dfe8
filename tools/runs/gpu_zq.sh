#!/bin/bash
# zquant timing on the GPU box: parity tests of the step-4 kernels, then the
# microbenchmark (q16 source) under timing knobs.
set -e
mkdir -p gpurun_out/zq1
timeout -k 10 300 python -u -m pytest tests/test_gpu_depth16.py tests/test_gpu_streamed.py tests/test_gpu_zq16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/zq1/pytest.log 2>&1
tail -1 gpurun_out/zq1/pytest.log
timeout -k 10 300 python -u tools/bench_zquant.py --q16 --groups 1 --reps 3 > gpurun_out/zq1/q16.log 2>&1
grep full16 gpurun_out/zq1/q16.log
