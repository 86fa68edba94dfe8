#!/bin/bash
# Quad-row LDS image for k_gram8: Gram parity tests, then A/B timing vs the pair-row image.
set -e
O=gpurun_out/ql; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gram or knn" > $O/pytest.log 2>&1
echo "pytest: $(tail -1 $O/pytest.log)"
timeout -k 10 300 python -u tools/bench_gram.py --reps 3 --variants "kb21,kb21:QL=0,kb22,kb22:QL=0,kb26,kb26:QL=0" > $O/gram.log 2>&1
cat $O/gram.log
