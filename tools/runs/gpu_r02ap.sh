#!/bin/bash
# Round pass on the final tree (tests, smoke, bench, rocprof stats, PMC traffic) and the
# config-3 line (50k x 3M, streamed).
set -e
bash tools/gpu_round.sh r02ap
O=gpurun_out/r02ap
timeout -k 10 500 python3 -u bench.py --samples 50000 --steps 1 --warmup 1 --cpu-samples 2048 > $O/bench_cfg3.json 2> $O/bench_cfg3.err
python -c "import json; d=json.load(open('$O/bench_cfg3.json')); print('cfg3', d['ms_per_step'], d['stages_ms'], d['roofline']['frac'])"
