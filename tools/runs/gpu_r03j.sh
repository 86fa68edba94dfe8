#!/bin/bash
# round 3: device writer with parallel pwrite; from-files config 2 with the ingest trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gzwrite.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 &&
GRID_INGEST_TRACE=1 timeout -k 10 700 python -u tools/e2e_files.py --bgzf --device-ingest --json $O/e2e_dev.json > $O/e2e_dev.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
tail -n 3 $O/pytest.log; grep "ingest\]" $O/e2e_dev.log | head -60; tail -n 22 $O/e2e_dev.log | grep "e2e\]"
exit $rc
