#!/bin/bash
# Column statistics on the compact matrix: columns per thread (GRID_COL16_VW 2/4/8 = 4/8/16-B loads),
# bench stage times, then the compact-depth GPU parity tests under VW=8.
set -e
O=gpurun_out/colvw; mkdir -p $O
for v in 2 4 8; do
  GRID_COL16_VW=$v timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/vw$v.json 2> $O/vw$v.err
  echo "VW $v: $(python -c "import json; d=json.load(open('$O/vw$v.json')); print(d['ms_per_step'], d['stages_ms']['col_stats'])")"
done
GRID_COL16_VW=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_depth16.py tests/test_gpu_streamed.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest VW=8: $(tail -1 $O/pytest.log)"
