#!/bin/bash
# round 5: the pipelined ingest batches ramp up (512 MB, 1 GB, 2 GB, then 4 GB) and the pageable staging is mapped
# at its bound: ingest and e2e GPU tests, then config 2 from files at threads 16 / 4 / 1 (digests compared)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05au
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
RUN=r05au bash tools/runs/gpu_r05ah.sh
