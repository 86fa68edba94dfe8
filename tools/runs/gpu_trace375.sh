#!/bin/bash
# Kernel trace of the 1/8-bins shard step (per-rank work of the 8-GPU run): host gaps between kernels.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace375; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -- python3 $R/bench.py --bins 375000 --steps 10 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1
echo ok
