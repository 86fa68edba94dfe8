#!/bin/bash
# round 4: the device ingest's input/text buffers cached on the device context -- ingest / e2e tests, then
# from-files config 2 twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ac
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_gpu_e2e.py tests/test_gpu_gzwrite.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
  keep=--reuse; [ $r = 2 ] && keep=""
  GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/e2e_files.py --bgzf $keep --json $O/e2e_$r.json \
    > $O/e2e_$r.log 2>&1 || { tail -n 30 $O/e2e_$r.log; exit 1; }
  python -c "import json; d=json.load(open('$O/e2e_$r.json')); p=d['phases_s']; print('run $r', round(d['steps_4_7_s'],2), 'ingest', round(p['step4_ingest'],2), 'write', round(p['step4_write_text'],2), d['outputs_xxh3_64']['normalized.tsv.gz'], d['outputs_xxh3_64']['haploid.tsv'])"
  grep -h "batches done\|finish buffers\|finish done\|device ingest returned" $O/e2e_$r.log
done
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
