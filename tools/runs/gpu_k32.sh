#!/bin/bash
# Timing A/B only (tools build): half-split ring on a 32-wide K-blocked panel (QL=3) vs the
# half-split ring on the 64-wide panel (QL=2) vs the quad-row default (QL=1).  bench_gram's
# tile check compares each production variant's first tiles with a float64 product.
set -e
O=gpurun_out/k32; mkdir -p $O
timeout -k 10 300 python -u tools/bench_gram.py --reps 3 --variants "kb21:QL=3,kb21:QL=1,kb21:QL=2,kb26:QL=3,kb26:QL=1,kb22:QL=3,kb22:QL=1" > $O/gram.log 2>&1
cat $O/gram.log
timeout -k 10 400 python -u tools/bench_gram.py --n 50000 --k 386048 --reps 2 --variants "kb21:QL=3,kb21:QL=1" > $O/gram50k.log 2>&1
cat $O/gram50k.log
