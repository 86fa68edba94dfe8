#!/bin/bash
# Column statistics width at the 1/8-bins shard (per-rank work of the 8-GPU run): GRID_COL16_VW 1 / 2 / 4.
set -e
O=gpurun_out/col375; mkdir -p $O
for v in 1 2 4 1 2; do
  GRID_COL16_VW=$v timeout -k 10 200 python -u bench.py --bins 375000 --steps 10 --warmup 2 --no-cpu-baseline > $O/vw$v.json 2> $O/vw$v.err
  echo "VW $v: $(python -c "import json; d=json.load(open('$O/vw$v.json')); print(d['ms_per_step'], d['stages_ms']['col_stats'], d['stages_ms']['row_means'])")"
done
