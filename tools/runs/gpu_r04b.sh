#!/bin/bash
# round 4: device-ingest guard (host-inflated text CRC in HBM), native-error hand-over, ingest tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_gpu_inflate.py > $O/pytest.log 2>&1
rc=$?
tail -n 5 $O/pytest.log
exit $rc
