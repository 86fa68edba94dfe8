#!/bin/bash
# round 5: radix-select histograms with wave-aggregated LDS atomics: the selection / scale / sharded GPU tests,
# the one-GPU bench line and the per-rank step (bench --sim-world 8)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05bb
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_select.py tests/test_gpu_scale.py tests/test_gpu_sharded.py tests/test_gpu_kernels.py \
  > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
B="python -u bench.py --no-cpu-baseline --no-files-baseline --no-files-config2 --config3-steps 0"
timeout -k 10 300 $B --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -n 30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['stages_ms'])"
for r in 1 2; do
  timeout -k 10 200 $B --steps 20 --warmup 2 --sim-world 8 --sim-rank 0 > $O/sim_$r.json 2> $O/sim_$r.err \
    || { tail -n 30 $O/sim_$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sim_$r.json'));print('cfg2 rank', d['ms_per_step'], d['stages_ms'])"
done
