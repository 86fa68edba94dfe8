#!/bin/bash
# round 5: Gram tile-group size at config 2 (3,202 x 2.7 M): groups of GS < 32 tiles deal the
# cohort's 182 tiles to all eight XCDs over the full K range (KX=1), so every XCD streams the
# same K-steps at once (the panel's L2 misses shared in the Infinity Cache), against the cost
# model's K split
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ar
mkdir -p $O
timeout -k 10 500 python -u tools/bench_gram.py --n 3202 --k 2700000 --reps 5 \
  --variants kb21,kb21:KX=1:GS=23,kb21:KX=1:GS=24,kb21:KX=2:GS=23,kb21:KX=1:GS=12,kb21:KX=8,kb21:KX=2 \
  > $O/gram_gs_sweep.log 2>&1 || { tail -n 30 $O/gram_gs_sweep.log; exit 1; }
grep "min\|MISMATCH\|DIFFERENT" $O/gram_gs_sweep.log
