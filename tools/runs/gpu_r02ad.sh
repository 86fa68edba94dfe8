#!/bin/bash
# Per-rank shard sizes of the 2/4/8-GPU strong-scaling runs on one GPU (config 2 with 1/2, 1/4, 1/8 of the
# bins) and the config-3 line (50k x 3M, streamed), on the current tree.
set -e
O=gpurun_out/r02ad; mkdir -p $O
for b in 1500000 750000 375000; do
  timeout -k 10 200 python -u bench.py --bins $b --steps 10 --warmup 2 --no-cpu-baseline > $O/b$b.json 2> $O/b$b.err
  echo "bins $b: $(python -c "import json; d=json.load(open('$O/b$b.json')); print(d['ms_per_step'], d['stages_ms'])")"
done
timeout -k 10 500 python3 -u bench.py --samples 50000 --steps 1 --warmup 1 --cpu-samples 2048 > $O/bench_cfg3.json 2> $O/bench_cfg3.err
python -c "import json; d=json.load(open('$O/bench_cfg3.json')); print('cfg3', d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
