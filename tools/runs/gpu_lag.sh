#!/bin/bash
# k_gram8 pacing knobs with the dynamic unit counter: round lag and spin bound, config 2 and the 1/8 shard.
set -e
O=gpurun_out/lag; mkdir -p $O
for k in 2700000 337500; do
  timeout -k 10 250 python -u tools/bench_gram.py --k $k --reps 3 --variants "kb21,kb21:LAG=0,kb21:LAG=2,kb21:LAG=3,kb21:SPIN=0,kb21:SPIN=100000" > $O/k$k.log 2>&1
  echo "K $k"; grep min $O/k$k.log
done
