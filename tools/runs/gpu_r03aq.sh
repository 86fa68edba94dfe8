#!/bin/bash
# round 3, final tree, short: the GPU inflate / device ingest / e2e tests with the 2^8 inflate fast table
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03aq
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_ingest.py tests/test_gpu_e2e.py tests/test_gpu_gzwrite.py > $O/pytest.log 2>&1
rc=$?
tail -n 3 $O/pytest.log
exit $rc
