#!/bin/bash
# round 3: k_gram8 with 16x16x32 MFMAs (LAY 4, GRID_GRAM_Q16 A/B in the tools build) vs the
# production 32x32x16 ring at config 2 and at the config-3 chunk; whole-Gram equality vs production
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ae
mkdir -p $O
timeout -k 10 240 python -u tools/bench_gram.py --variants kb21,kb21:Q16=1,kb26,kb26:Q16=1,kb22,kb22:Q16=1 --reps 4 \
  > $O/gram_q16_ab_config2.log 2>&1 && cat $O/gram_q16_ab_config2.log &&
timeout -k 10 300 python -u tools/bench_gram.py --n 50000 --k 386048 --variants kb21,kb21:Q16=1 --reps 3 \
  > $O/gram_q16_ab_50k.log 2>&1 && cat $O/gram_q16_ab_50k.log
