#!/bin/bash
# round 6: every GPU test on the tree with the distributed drop-in, then the bench's N > 1 launch path
# rehearsed on this one GPU (2 and 4 gloo ranks sharing it; reduced cohort): rank 0 writes the cohort, the
# ranks run the distributed `grid wgs` K times, then the device chain
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests \
  > $O/pytest_gpu_full.log 2>&1 || { tail -n 60 $O/pytest_gpu_full.log; exit 1; }
tail -n 2 $O/pytest_gpu_full.log
for w in 2 4; do
  GRID_BENCH_SHARE_GPU=1 GRID_DIST_BACKEND=gloo timeout -k 10 240 python -u bench.py --gpus $w --samples 512 \
    --bins 400000 --steps 2 --warmup 1 --no-cpu-baseline --config3-steps 0 --headline files \
    > $O/gloo_w${w}_files.json 2> $O/gloo_w${w}_files.err || { tail -n 40 $O/gloo_w${w}_files.err; exit 1; }
  python -c "import json;d=json.load(open('$O/gloo_w${w}_files.json'));print('w$w', d['n_gpus'], d['value'], d['ms_per_step'], d['from_files']['stages_s'], d['device_chain']['ms_per_step'])"
done
