#!/bin/bash
# round 4: two phasing lanes (one per dipCN buffer) -- the chain tests that run Steps47, smoke, then the bench
# at the 1/8-bins per-rank shape and at config 2 with 5 and 20 timed steps (the end-of-run phasing tail)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sharded.py tests/test_gpu_zq16.py tests/test_gpu_depth16.py tests/test_gpu_streamed.py \
  tests/test_gpu_scale.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok"
for a in "375000 10" "375000 20" "3000000 5" "3000000 20"; do
  set -- $a
  timeout -k 10 250 python -u bench.py --bins $1 --steps $2 --warmup 2 --no-cpu-baseline --config3-steps 0 \
    --no-files-config2 > $O/bench_b$1_s$2.json 2> $O/bench_b$1_s$2.err || { tail -n 20 $O/bench_b$1_s$2.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_b$1_s$2.json')); print('bins', $1, 'steps', $2, round(d['ms_per_step'],3), d['stages_ms'])"
done
