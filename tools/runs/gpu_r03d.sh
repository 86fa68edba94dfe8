#!/bin/bash
# round 3: device inflate + device mosdepth ingest tests, inflate throughput, e2e goldens
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_inflate.py tests/test_gpu_ingest.py tests/test_gpu_configs.py::test_streamed_property_checks_small tests/test_gpu_e2e.py > gpurun_out/r03d_tests.log 2>&1
rc=$?
timeout -k 10 300 python -u tools/bench_inflate.py --files 64 --distinct 8 --json gpurun_out/r03d_inflate_bench.json > gpurun_out/r03d_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_inflate.py --files 64 --distinct 8 --bgzf --json gpurun_out/r03d_inflate_bench_bgzf.json >> gpurun_out/r03d_bench.log 2>&1
rc2=$?
tail -3 gpurun_out/r03d_tests.log gpurun_out/r03d_bench.log
exit $(( rc | rc2 ))
