#!/bin/bash
# Config-3 (50k x 3M) HBM traffic per Gram launch (FETCH_SIZE / WRITE_SIZE passes) and an N=2
# self-launched rehearsal (ranks share the one GPU, gloo) on the current tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02al
mkdir -p $O
cd $R
GRID_BENCH_SHARE_GPU=1 GRID_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/bench_n2_share.json 2> $O/bench_n2_share.err
rc=$?; echo "n2 rc=$rc"; tail -1 $O/bench_n2_share.json | cut -c1-200; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --samples 50000 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/pmc_fetch -- python3 $B > $O/pmc_fetch.log 2>&1
echo "pmc fetch rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/pmc_write -- python3 $B > $O/pmc_write.log 2>&1
echo "pmc write rc=$?"
