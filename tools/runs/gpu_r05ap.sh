#!/bin/bash
# round 5, final pass of the tree: GPU tests, smoke, the default bench line (all its records), kernel stats and the
# two PMC traffic passes (device chain), then the multi-rank launcher rehearsed on this one GPU (gloo, ranks sharing
# it; reduced shape) for both Gram splits, and RCCL at world 1
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r05ap}
mkdir -p $O
cd $R
bash tools/runs/gpu_r05n.sh.inner $O || exit 1
