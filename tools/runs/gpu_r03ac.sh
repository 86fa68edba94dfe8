#!/bin/bash
# round 3: the driver's N > 1 launch path rehearsed on one GPU -- bench.py --gpus 2 self-launching
# torch.distributed.run, ranks sharing the GPU over gloo (RCCL refuses two ranks on one GPU);
# checks that stdout carries exactly one JSON line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ac
mkdir -p $O
GRID_BENCH_SHARE_GPU=1 GRID_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --bins 375000 --steps 3 --warmup 1 \
  --no-cpu-baseline --config3-steps 0 > $O/n2_stdout.txt 2> $O/n2_stderr.txt
rc=$?
echo "rc=$rc lines=$(wc -l < $O/n2_stdout.txt)"
python -c "
import json; L=open('$O/n2_stdout.txt').read().splitlines(); d=json.loads(L[0]); print(len(L), d['n_gpus'], d['ms_per_step'], d['config']['workload'])"
tail -n 5 $O/n2_stderr.txt
exit $rc
