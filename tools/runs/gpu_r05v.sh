#!/bin/bash
# round 5: Gram schedule sweep at the per-rank shape (3,202 x 331,775: config 2 over 8 bin shards) -- K ranges
# (KX), chunks (KC) and the unit price (UF) of the cost model, against its own choice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 400 python -u tools/bench_gram.py --n 3202 --k 331775 --reps 5 \
  --variants kb21,kb21:KX=1,kb21:KX=2,kb21:KX=4,kb21:KX=8,kb21:UF=10,kb21:UF=20,kb21:UF=80,kb21:UF=160,kb21:DYN=0 \
  > $O/gram_rank_sweep.log 2>&1 || { tail -n 30 $O/gram_rank_sweep.log; exit 1; }
grep "min" $O/gram_rank_sweep.log
