#!/bin/bash
# round 3: device gzip inflate (tests + throughput), then the -m gpu suite minus the two long configs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_inflate.py tests/test_gpu_configs.py::test_streamed_property_checks_small > gpurun_out/r03c_inflate.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_inflate.py --files 64 --distinct 8 --json gpurun_out/r03c_inflate_bench.json > gpurun_out/r03c_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_inflate.py --files 64 --distinct 8 --bgzf --json gpurun_out/r03c_inflate_bench_bgzf.json >> gpurun_out/r03c_bench.log 2>&1 &&
timeout -k 10 1500 $T tests -m gpu --deselect tests/test_gpu_configs.py::test_config3_50k_x_3M_streamed \
  --deselect tests/test_gpu_configs.py::test_config4_50k_x_30M_streamed --deselect tests/test_gpu_inflate.py \
  > gpurun_out/r03c_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/r03c_inflate.log gpurun_out/r03c_bench.log gpurun_out/r03c_pytest.log
exit $rc
