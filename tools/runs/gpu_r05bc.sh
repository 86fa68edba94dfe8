#!/bin/bash
# round 5: the 8-rank launcher rehearsed on this one GPU (gloo, 8 ranks sharing it; reduced shape) for both Gram
# splits -- the driver's N = 8 path end to end, bit-identical results checked by the tests elsewhere
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05bc
mkdir -p $O
for s in bin cohort; do
  GRID_BENCH_SHARE_GPU=1 GRID_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 8 --shard $s --samples 1024 \
    --bins 400000 --steps 2 --warmup 1 --no-cpu-baseline --no-files-baseline --no-files-config2 --config3-steps 0 \
    > $O/gloo_w8_$s.json 2> $O/gloo_w8_$s.err || { tail -n 30 $O/gloo_w8_$s.err; exit 1; }
  python -c "import json;d=json.load(open('$O/gloo_w8_$s.json'));print('gloo w8 $s', d['n_gpus'], d['ms_per_step'], d['value'], d['config']['parallelism'])"
done
