#!/bin/bash
# k_gram8 dynamic unit counter (GRID_GRAM_DYN): Gram parity tests, A/B alone and inside the 1/8-bins
# shard step (where the phasing lane's kernel holds one CU when the Gram launches).
set -e
O=gpurun_out/dyn; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gram or knn" > $O/pytest.log 2>&1
echo "pytest: $(tail -1 $O/pytest.log)"
timeout -k 10 200 python -u tools/bench_gram.py --k 337500 --reps 3 --variants "kb21:DYN=0,kb21:DYN=1" > $O/g337.log 2>&1
grep min $O/g337.log
timeout -k 10 200 python -u tools/bench_gram.py --reps 3 --variants "kb21:DYN=0,kb21:DYN=1" > $O/g27.log 2>&1
grep min $O/g27.log
for d in 0 1 0 1; do
  GRID_GRAM_DYN=$d timeout -k 10 200 python -u bench.py --bins 375000 --steps 10 --warmup 2 --no-cpu-baseline > $O/b375_$d.json 2> $O/b375_$d.err
  echo "bins 375000 DYN=$d: $(python -c "import json; d=json.load(open('$O/b375_$d.json')); print(d['ms_per_step'], d['stages_ms']['zquant_gram'])")"
done
for d in 0 1; do
  GRID_GRAM_DYN=$d timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/b3m_$d.json 2> $O/b3m_$d.err
  echo "bins 3M DYN=$d: $(python -c "import json; d=json.load(open('$O/b3m_$d.json')); print(d['ms_per_step'], d['stages_ms']['zquant_gram'])")"
done
