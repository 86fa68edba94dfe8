#!/bin/bash
# round 4: the 8-wave inflate in the product library -- inflate / ingest / e2e tests, then from-files config 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_ingest.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 \
  || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
GRID_INGEST_TRACE=1 timeout -k 10 600 python -u tools/e2e_files.py --bgzf --json $O/e2e_files_config2_bgzf.json \
  > $O/e2e.log 2>&1 || { tail -n 30 $O/e2e.log; exit 1; }
grep -E "e2e\] .*(step4_ingest|step4_write|done in)" $O/e2e.log | tail -n 8
python -c "import json; d=json.load(open('$O/e2e_files_config2_bgzf.json')); print(d['steps_4_7_s'], d['outputs_xxh3_64'])"
