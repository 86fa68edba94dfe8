#!/bin/bash
# k_gram8 timing probes on the quad-row image: 3202 x 2.7M and one config-3 chunk (50k x 386k)
set -e
O=gpurun_out/ql2; mkdir -p $O
timeout -k 10 300 python -u tools/bench_gram.py --reps 3 --variants "kb21,kb24,kb25,kb26,kb22" > $O/gram3202.log 2>&1
cat $O/gram3202.log
timeout -k 10 400 python -u tools/bench_gram.py --n 50000 --k 386048 --reps 2 --variants "kb21,kb21:QL=0,kb24,kb26,kb22" > $O/gram50k.log 2>&1
cat $O/gram50k.log
timeout -k 10 300 python -u tools/bench_zquant.py --q16 --reps 3 --env "GRID_Z7_PROBE=0;GRID_Z7_PROBE=1;GRID_Z7_PROBE=2;GRID_Z7_PROBE=3;GRID_Z7_PROBE=4;GRID_Z7_PROBE=7" > $O/zq.log 2>&1
cat $O/zq.log
