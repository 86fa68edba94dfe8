#!/bin/bash
# round 5: the host-to-device copies staged through a page-locked ring by 8 threads: ingest tests, then traced
# from-files config 2 at threads 16, 4 and 1 on one generated cohort
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
D=/dev/shm/grid_r05l
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --generate-only --reuse > $O/gen.log 2>&1 \
  || { tail -n 20 $O/gen.log; exit 1; }
for t in 16 4 1; do
  GRID_INGEST_TRACE=1 timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --reuse --threads $t \
    --json $O/e2e_t$t.json > $O/e2e_t$t.log 2>&1 || { tail -n 30 $O/e2e_t$t.log; rm -rf $D; exit 1; }
  grep "batch .* enqueued" $O/e2e_t$t.log | head -6
  python -c "import json; d=json.load(open('$O/e2e_t$t.json')); print('threads $t', round(d['steps_4_7_s'],2), {k: round(v,2) for k,v in d['phases_s'].items() if k.startswith('step4') or k.startswith('release')}, d['outputs_xxh3_64'])"
done
rm -rf $D
