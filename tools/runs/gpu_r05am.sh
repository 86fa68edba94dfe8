#!/bin/bash
# round 5: the ingest's parse on its own stream (batch b's parse beside batch b+1's inflate, text double-buffered):
# ingest / e2e / inflate GPU tests, then from files at config 2, threads 16 / 4 / 1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${RUN:-r05am}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_gpu_e2e.py tests/test_gpu_inflate.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
RUN=${RUN:-r05am} bash tools/runs/gpu_r05ah.sh
