#!/bin/bash
# k_zquant7 16-B loads (GRID_Z7_W16): timing A/B, then the zquant / chain GPU parity tests under W16=1.
set -e
O=gpurun_out/w16; mkdir -p $O
timeout -k 10 300 python -u tools/bench_zquant.py --q16 --reps 3 --env "GRID_Z7_W16=0;GRID_Z7_W16=1;GRID_Z7_W16=1,GRID_Z7_PROBE=3;GRID_Z7_W16=0,GRID_Z7_PROBE=3" > $O/zq.log 2>&1
cat $O/zq.log
GRID_Z7_W16=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_depth16.py tests/test_gpu_zq16.py tests/test_gpu_scale.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest W16=1: $(tail -1 $O/pytest.log)"
