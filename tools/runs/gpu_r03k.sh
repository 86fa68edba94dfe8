#!/bin/bash
# round 3: from-files config 2 after the one-listing file lookup: BGZF and plain-gzip cohorts, device ingest
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 &&
GRID_INGEST_TRACE=1 timeout -k 10 500 python -u tools/e2e_files.py --bgzf --device-ingest --json $O/e2e_bgzf_dev.json > $O/e2e_bgzf_dev.log 2>&1 &&
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out &&
GRID_INGEST_TRACE=1 timeout -k 10 500 python -u tools/e2e_files.py --device-ingest --json $O/e2e_plain_dev.json > $O/e2e_plain_dev.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
tail -n 3 $O/pytest.log; for f in $O/e2e_bgzf_dev.log $O/e2e_plain_dev.log; do grep "e2e\]" $f | grep -v files | tail -n 14; grep "ingest\] batch 1:" $f; done
exit $rc
