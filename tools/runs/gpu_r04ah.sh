#!/bin/bash
# round 4, final tree: bench.py --gpus 8 and --gpus 2 rehearsed on the one GPU over gloo (ranks share it),
# reduced shape for 8 ranks, config 2's shape for 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ah
mkdir -p $O
GRID_BENCH_SHARE_GPU=1 GRID_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 8 --steps 3 --warmup 1 \
  --samples 1024 --bins 524288 --hbm-budget-gb 20 --no-cpu-baseline --config3-steps 0 \
  > $O/bench_gpus8_share.json 2> $O/bench_gpus8_share.err || { tail -n 30 $O/bench_gpus8_share.err; exit 1; }
python -c "import json; L=open('$O/bench_gpus8_share.json').read().splitlines(); assert len(L)==1, L; d=json.loads(L[0]); print('gpus8', d['n_gpus'], round(d['value']), round(d['ms_per_step'],2))"
GRID_BENCH_SHARE_GPU=1 GRID_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 3 --warmup 1 \
  --hbm-budget-gb 100 --no-cpu-baseline --config3-steps 0 \
  > $O/bench_gpus2_share.json 2> $O/bench_gpus2_share.err || { tail -n 30 $O/bench_gpus2_share.err; exit 1; }
python -c "import json; L=open('$O/bench_gpus2_share.json').read().splitlines(); assert len(L)==1, L; d=json.loads(L[0]); print('gpus2', d['n_gpus'], round(d['value']), round(d['ms_per_step'],2), d['config']['workload'])"
