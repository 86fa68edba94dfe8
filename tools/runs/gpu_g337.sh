#!/bin/bash
# k_gram8 at the per-rank K of the 8-GPU run (337.5k) and at config 2: K-blocked (K32, half-split ring)
# vs row-major panels (quad-row / half-split images).
set -e
O=gpurun_out/g337; mkdir -p $O
for k in 337500 2700000; do
  timeout -k 10 200 python -u tools/bench_gram.py --k $k --reps 3 --variants "kb21,21,21:QL=2,kb21:UF=10,kb21:UF=100" > $O/k$k.log 2>&1
  echo "K $k"; grep min $O/k$k.log
done
