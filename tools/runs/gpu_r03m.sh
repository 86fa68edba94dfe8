#!/bin/bash
# round 3: step path without torch (pinned staging via the ABI), device ingest on by default;
# e2e goldens on both ingest paths; from-files config 2 (BGZF) with timestamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_e2e.py tests/test_gpu_ingest.py tests/test_gpu_gzwrite.py tests/test_gpu_inflate.py > $O/pytest.log 2>&1 &&
GRID_INGEST_TRACE=1 timeout -k 10 500 python -u tools/e2e_files.py --bgzf --json $O/e2e_bgzf_dev.json > $O/e2e_bgzf_dev.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
tail -n 3 $O/pytest.log; grep -v "batch files" $O/e2e_bgzf_dev.log | grep "ingest\]\|e2e\]" | grep -v " files$" | tail -n 40
exit $rc
