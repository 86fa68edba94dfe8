#!/bin/bash
# round 3: device gzip writer -- its tests + the e2e goldens, then from-files config 2 with it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gzwrite.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 &&
timeout -k 10 700 python -u tools/e2e_files.py --bgzf --device-ingest --json $O/e2e_dev.json > $O/e2e_dev.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
tail -n 15 $O/pytest.log; tail -n 22 $O/e2e_dev.log | cut -c1-400
exit $rc
