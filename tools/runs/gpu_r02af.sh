#!/bin/bash
# Config-4 bench line (50k x 30M bins, bin-streamed, 1 GPU) on the current tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02af
mkdir -p $O
cd $R
timeout -k 10 700 python3 -u bench.py --samples 50000 --bins 30000000 --steps 1 --warmup 1 --cpu-samples 2048 \
  > $O/bench_cfg4.json 2> $O/bench_cfg4.err
rc=$?; echo "cfg4 rc=$rc"; cat $O/bench_cfg4.json
