#!/bin/bash
# round 3: device ingest, copy stream -> parse stream ordering (grid_stream_after); control arm without it, then
# every device-ingest test with it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ag
mkdir -p $O
timeout -k 10 200 python -u tools/runs/xstream_probe.py > $O/control_no_wait.log 2>&1
echo "control arm (no wait) rc=$?"; tail -n 4 $O/control_no_wait.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_gpu_inflate.py > $O/pytest_ingest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest_ingest.log | tail -n 40; tail -n 3 $O/pytest_ingest.log
exit $rc
