#!/bin/bash
# N=2 self-launched bench rehearsal on the compact-depth default (ranks share
# the one GPU, gloo) and a config-3 line (50k x 3M, streamed int32 chunks).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02s
mkdir -p $O
cd $R
GRID_BENCH_SHARE_GPU=1 GRID_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/bench_n2_share.json 2> $O/bench_n2_share.err
rc=$?; echo "n2 rc=$rc"; cat $O/bench_n2_share.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py --samples 50000 --steps 1 --warmup 1 --cpu-samples 2048 \
  > $O/bench_cfg3.json 2> $O/bench_cfg3.err
rc=$?; echo "cfg3 rc=$rc"; cat $O/bench_cfg3.json
