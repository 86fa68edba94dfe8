#!/bin/bash
# round 3: u32 fast tables (4 waves/CU), member-granular launches, CPU/GPU split ingest
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_inflate.py tests/test_gpu_ingest.py > gpurun_out/r03f_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_inflate.py --files 64 --distinct 8 --json gpurun_out/r03f_inflate_64.json > gpurun_out/r03f_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_inflate.py --files 1024 --distinct 8 --bgzf --units --json gpurun_out/r03f_inflate_1024_units.json >> gpurun_out/r03f_bench.log 2>&1 &&
GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/bench_dev_ingest.py --samples 256 --json gpurun_out/r03f_dev_ingest_256.json >> gpurun_out/r03f_bench.log 2>&1
rc=$?
tail -n 4 gpurun_out/r03f_tests.log
tail -n 12 gpurun_out/r03f_bench.log
exit $rc
