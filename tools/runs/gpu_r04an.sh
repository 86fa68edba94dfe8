#!/bin/bash
# round 4, final tree: the per-rank 1/8-bins step (3,202 x 375,000) with 20 timed steps, twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04an
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --bins 375000 --steps 20 --warmup 2 --no-cpu-baseline --config3-steps 0 \
    --no-files-config2 > $O/bench_bins375000_$r.json 2> $O/bench_bins375000_$r.err || { tail -n 20 $O/bench_bins375000_$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_bins375000_$r.json')); print('run $r', round(d['ms_per_step'],3), d['stages_ms'])"
done
