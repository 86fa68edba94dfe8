#!/bin/bash
# Synthetic cohort generator with 16-B stores: GPU tests that consume it, then the config-3 line.
set -e
O=gpurun_out/synth; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_depth16.py tests/test_gpu_zq16.py tests/test_gpu_streamed.py tests/test_gpu_scale.py tests/test_gpu_sharded.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest: $(tail -1 $O/pytest.log)"
timeout -k 10 500 python3 -u bench.py --samples 50000 --steps 1 --warmup 1 --cpu-samples 2048 > $O/bench_cfg3.json 2> $O/bench_cfg3.err
python -c "import json; d=json.load(open('$O/bench_cfg3.json')); print(d['ms_per_step'], d['stages_ms'])"
