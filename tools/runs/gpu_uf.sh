#!/bin/bash
# Gram unit-flush cost in the (kx, kc) choice: K ranges of the strong-scaling shards
set -e
O=gpurun_out/uf; mkdir -p $O
for k in 337500 675000 1350000 2700000; do
  timeout -k 10 200 python -u tools/bench_gram.py --k $k --reps 3 --variants "kb21:UF=0,kb21:UF=20,kb21:UF=40,kb21:UF=80" > $O/k$k.log 2>&1
  echo "K $k"; grep min $O/k$k.log
done
for b in 1500000 750000 375000; do
  timeout -k 10 200 python -u bench.py --bins $b --steps 10 --warmup 2 --no-cpu-baseline > $O/b$b.json 2> $O/b$b.err
  echo "bins $b"; cat $O/b$b.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'])"
done
