#!/bin/bash
# Half-split ring (LAY 2) for k_gram8: Gram parity tests, then A/B vs the quad-row (1) and pair-row (0) images.
set -e
O=gpurun_out/qh; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gram or knn" > $O/pytest.log 2>&1
echo "pytest: $(tail -1 $O/pytest.log)"
timeout -k 10 300 python -u tools/bench_gram.py --reps 3 --variants "kb21,kb21:QL=1,kb21:QL=0,kb26,kb26:QL=1,kb22" > $O/gram.log 2>&1
cat $O/gram.log
timeout -k 10 400 python -u tools/bench_gram.py --n 50000 --k 386048 --reps 2 --variants "kb21,kb21:QL=1" > $O/gram50k.log 2>&1
cat $O/gram50k.log
