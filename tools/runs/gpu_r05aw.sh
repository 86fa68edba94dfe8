#!/bin/bash
# round 5: pipelined ingest batch size (GRID_INGEST_BATCH_MB 4096 / 2048 / 1024, the ramp below it) at config 2
# from files, threads 16, host-side batch times on stderr; output digests compared
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05aw
mkdir -p $O
export TMPDIR=/tmp
D=/dev/shm/grid_r05aw
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --generate-only --reuse > $O/gen.log 2>&1 \
  || { tail -n 20 $O/gen.log; rm -rf $D; exit 1; }
for mb in 4096 2048 1024 2048 4096 1024; do
  GRID_INGEST_BATCH_MB=$mb GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/e2e_files.py --bgzf --data $D --reuse \
    --threads 16 --json $O/e2e_b$mb.json > $O/e2e_b$mb.log 2>&1 || { tail -n 30 $O/e2e_b$mb.log; rm -rf $D; exit 1; }
  python -c "import json; d=json.load(open('$O/e2e_b$mb.json')); print('batch MB $mb', round(d['steps_4_7_s'],2), round(d['phases_s']['step4_ingest'],3), d['outputs_xxh3_64'].get('normalized.tsv.gz'), d['outputs_xxh3_64'].get('neighbors.zMax2.0.tsv.gz'))"
done
rm -rf $D
