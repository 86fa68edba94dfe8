#!/bin/bash
# round 3: device-resident selection vs the host-synchronising entry points (edge cases)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ad
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_select.py > $O/pytest.log 2>&1
rc=$?
tail -n 15 $O/pytest.log
exit $rc
