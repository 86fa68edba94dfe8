#!/bin/bash
# Per-rank work of the strong-scaling runs on one GPU: config 2 with 1/2, 1/4, 1/8 of the bins
set -e
O=gpurun_out/shardsim; mkdir -p $O
for b in 1500000 750000 375000; do
  timeout -k 10 200 python -u bench.py --bins $b --steps 10 --warmup 2 --no-cpu-baseline > $O/b$b.json 2> $O/b$b.err
  echo "bins $b"; cat $O/b$b.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -- python3 $GRAFT_REPO_ROOT/bench.py --bins 375000 --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/stats.log 2>&1
echo stats ok
