#!/bin/bash
# round 4: pipelined BGZF ingest batches -- ingest/inflate GPU tests, then the from-files config-2 run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_gpu_inflate.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 3 $O/pytest.log
GRID_INGEST_TRACE=1 timeout -k 10 600 python -u tools/e2e_files.py --bgzf --json $O/e2e_files_config2_bgzf.json \
  > $O/e2e.log 2>&1
rc=$?
grep -E "ingest\]|e2e\]" $O/e2e.log | tail -n 30
exit $rc
