#!/bin/bash
# round 5: where the from-files ingest's time goes -- traced e2e runs at threads 16 and 4 (per-batch read times)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05i
mkdir -p $O
D=/dev/shm/grid_r05i
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --generate-only --reuse > $O/gen.log 2>&1 \
  || { tail -n 20 $O/gen.log; exit 1; }
for t in 16 4; do
  GRID_INGEST_TRACE=1 timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --reuse --threads $t \
    --json $O/e2e_t$t.json > $O/e2e_t$t.log 2>&1 || { tail -n 30 $O/e2e_t$t.log; rm -rf $D; exit 1; }
  grep "\[ingest\]" $O/e2e_t$t.log | head -12
  python -c "import json; d=json.load(open('$O/e2e_t$t.json')); print('threads $t', round(d['steps_4_7_s'],2), round(d['phases_s']['step4_ingest'],2))"
done
rm -rf $D
