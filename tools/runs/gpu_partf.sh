#!/bin/bash
# k_gram8 partial mode (plain int32 tile stores + per-tile reduction, GRID_GRAM_PART_MB): Gram parity
# tests, A/B vs int64 atomics, and the bench step (config 2 and the 1/8-bins shard).
set -e
O=gpurun_out/partf; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gram or knn or shard" > $O/pytest.log 2>&1
echo "pytest: $(tail -1 $O/pytest.log)"
for k in 2700000 337500; do
  timeout -k 10 200 python -u tools/bench_gram.py --k $k --reps 3 --variants "kb21:PART_MB=0,kb21,kb21:PART_MB=0,kb21" > $O/k$k.log 2>&1
  echo "K $k"; grep min $O/k$k.log
done
for p in 0 4096 0 4096; do
  GRID_GRAM_PART_MB=$p timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/b3m_$p.json 2> $O/b3m_$p.err
  echo "3M PART_MB=$p: $(python -c "import json; d=json.load(open('$O/b3m_$p.json')); print(d['ms_per_step'], d['stages_ms']['zquant_gram'])")"
done
for p in 0 4096; do
  GRID_GRAM_PART_MB=$p timeout -k 10 200 python -u bench.py --bins 375000 --steps 10 --warmup 2 --no-cpu-baseline > $O/b375_$p.json 2> $O/b375_$p.err
  echo "375k PART_MB=$p: $(python -c "import json; d=json.load(open('$O/b375_$p.json')); print(d['ms_per_step'], d['stages_ms']['zquant_gram'])")"
done
