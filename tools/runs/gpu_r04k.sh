#!/bin/bash
# round 4: the CPU-baseline sweep on the GPU box's host cores (no GPU use)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 1140 python -u tools/cpu_sweep.py --workers 6 --data /dev/shm/grid_sweep --json $O/cpu_sweep.json \
  > $O/cpu_sweep.out 2> $O/cpu_sweep.err
rc=$?
rm -rf /dev/shm/grid_sweep
tail -n 12 $O/cpu_sweep.err
exit $rc
