#!/bin/bash
# Column statistics with software-pipelined row groups (GRID_COL_PF): bench stage times, then the
# compact-depth GPU parity tests under PF=1.
set -e
O=gpurun_out/colpf; mkdir -p $O
for v in 0 1 0 1; do
  GRID_COL_PF=$v timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pf$v.json 2> $O/pf$v.err
  echo "PF $v: $(python -c "import json; d=json.load(open('$O/pf$v.json')); print(d['ms_per_step'], d['stages_ms']['col_stats'])")"
done
GRID_COL_PF=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_depth16.py tests/test_gpu_streamed.py tests/test_gpu_kernels.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest PF=1: $(tail -1 $O/pytest.log)"
