#!/bin/bash
# Column statistics rows in flight (GRID_COL16_CU=16 vs 8) at the 1/8 and 1/2 shards and at full width.
set -e
O=gpurun_out/cu16; mkdir -p $O
for b in 375000 1500000 3000000; do
  for c in 8 16; do
    if [ $c = 16 ]; then export GRID_COL16_CU=16; else unset GRID_COL16_CU; fi
    timeout -k 10 200 python -u bench.py --bins $b --steps 6 --warmup 2 --no-cpu-baseline > $O/b${b}_cu$c.json 2> $O/b${b}_cu$c.err
    echo "bins $b CU $c: $(python -c "import json; d=json.load(open('$O/b${b}_cu$c.json')); print(d['ms_per_step'], d['stages_ms']['col_stats'])")"
  done
done
unset GRID_COL16_CU
GRID_COL16_CU=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_depth16.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest CU16: $(tail -1 $O/pytest.log)"
