#!/bin/bash
# round 3: fast inflate loop -- inflate/ingest tests, throughput at 64 and 1024 files, plain and BGZF
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_inflate.py tests/test_gpu_ingest.py > gpurun_out/r03e_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_inflate.py --files 64 --distinct 8 --json gpurun_out/r03e_inflate_64.json > gpurun_out/r03e_bench.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_inflate.py --files 64 --distinct 8 --bgzf --json gpurun_out/r03e_inflate_64_bgzf.json >> gpurun_out/r03e_bench.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_inflate.py --files 1024 --distinct 8 --json gpurun_out/r03e_inflate_1024.json >> gpurun_out/r03e_bench.log 2>&1
rc=$?
tail -n 5 gpurun_out/r03e_tests.log gpurun_out/r03e_bench.log
exit $rc
