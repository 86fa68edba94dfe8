#!/bin/bash
# round 3: is k_gram8's L2 -> LDS feed bound per CU (in-flight bytes over latency) or shared
# (L2 / MALL / HBM)?  The DMA-only probe (kb26) and production on 32, 24, 16 and 8 workgroups per XCD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ak
mkdir -p $O
timeout -k 10 400 python -u tools/bench_gram.py --reps 2 \
  --variants kb26,kb26:PER=24,kb26:PER=16,kb26:PER=8,kb21,kb21:PER=24,kb21:PER=16,kb21:PER=8 > $O/gram_per_cu_sweep.log 2>&1
rc=$?
cat $O/gram_per_cu_sweep.log
exit $rc
