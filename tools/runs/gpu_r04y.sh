#!/bin/bash
# round 4: the pipelined batches' host share (GRID_INGEST_HOST_FRAC: every k-th BGZF file inflated by the host
# threads beside the GPU) -- the device-ingest tests, then from-files config 2 at fractions 0, 1/6, 1/4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --generate-only > $O/gen.log 2>&1 || { tail -n 20 $O/gen.log; exit 1; }
for f in 0.25 0.33 0.2 0.25 0.33; do
  GRID_INGEST_HOST_FRAC=$f GRID_INGEST_TRACE=1 timeout -k 10 300 python -u tools/e2e_files.py --bgzf --reuse \
    --json $O/e2e_h$f.json > $O/e2e_h$f.log 2>&1 || { tail -n 30 $O/e2e_h$f.log; exit 1; }
  python -c "import json; d=json.load(open('$O/e2e_h$f.json')); p=d['phases_s']; print('frac', '$f', round(d['steps_4_7_s'],2), 'ingest', round(p['step4_ingest'],2), 'write', round(p['step4_write_text'],2), d['outputs_xxh3_64']['normalized.tsv.gz'], d['outputs_xxh3_64']['haploid.tsv'])"
done
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
