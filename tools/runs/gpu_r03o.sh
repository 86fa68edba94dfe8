#!/bin/bash
# round 3: 8 KiB inflate ring (11 waves/CU, far matches from HBM) -- inflate/ingest tests, then
# the device ingest at 1024 BGZF files: cost-model split and GPU-only
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_ingest.py > $O/pytest.log 2>&1 &&
GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/bench_dev_ingest.py --samples 1024 --modes model,gpu --json $O/dev_ingest_1024.json > $O/dev_ingest.log 2>&1
rc=$?
rm -rf /dev/shm/grid_dev_ingest
tail -n 3 $O/pytest.log; grep -v "batch files" $O/dev_ingest.log | grep -v generated | tail -n 30
exit $rc
