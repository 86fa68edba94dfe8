#!/bin/bash
# round 4: the device writer's pwrite threads per batch (GRID_WRITER_W, tools build) on the box's disk --
# from-files config 2 with 4 (the default) and 8 threads, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --generate-only > $O/gen.log 2>&1 || { tail -n 20 $O/gen.log; exit 1; }
for w in 4 8 4 8 12; do
  GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so GRID_WRITER_W=$w timeout -k 10 300 python -u tools/e2e_files.py \
    --bgzf --reuse --json $O/e2e_w$w.json > $O/e2e_w$w.log 2>&1 || { tail -n 30 $O/e2e_w$w.log; exit 1; }
  python -c "import json; d=json.load(open('$O/e2e_w$w.json')); p=d['phases_s']; print('W $w', round(d['steps_4_7_s'],2), 'ingest', round(p['step4_ingest'],2), 'write', round(p['step4_write_text'],2), d['outputs_xxh3_64']['normalized.tsv.gz'])"
done
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
