#!/bin/bash
# round 5: from files at config 2 after the inflate rework (37 -> 63.6 GB/s): threads 16 / 4 / 1 on one generated
# cohort, output digests compared, the step-4 file read back (CRC-checked) at threads 16
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${RUN:-r05ah}
mkdir -p $O
export TMPDIR=/tmp
D=/dev/shm/grid_${RUN:-r05ah}
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --generate-only --reuse > $O/gen.log 2>&1 \
  || { tail -n 20 $O/gen.log; exit 1; }
for t in 16 4 1; do
  V=""; [ $t = 16 ] && V="--verify-normalized"
  timeout -k 10 400 python -u tools/e2e_files.py --bgzf --data $D --reuse --threads $t $V --json $O/e2e_t$t.json \
    > $O/e2e_t$t.log 2>&1 || { tail -n 30 $O/e2e_t$t.log; rm -rf $D; exit 1; }
  python -c "import json; d=json.load(open('$O/e2e_t$t.json')); print('threads $t', round(d['steps_4_7_s'],2), {k: round(v,2) for k,v in d['phases_s'].items() if k.startswith('step')}, d['outputs'].get('normalized.tsv.gz'), d.get('normalized_readback', {}).get('zq_xxh3_64'), d['outputs_xxh3_64'].get('neighbors.zMax2.0.tsv.gz'))"
done
rm -rf $D
