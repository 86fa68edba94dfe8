#!/bin/bash
# round 5: after the Gram's group-size parameter -- the Gram, scale, sharded and cohort-split GPU tests, then
# the default bench line (no from-files leg)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05as
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_scale.py tests/test_gpu_sharded.py tests/test_gpu_general_knn.py \
  > $O/pytest_gram.log 2>&1 || { tail -n 40 $O/pytest_gram.log; exit 1; }
tail -n 2 $O/pytest_gram.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-files-baseline --no-files-config2 --config3-steps 0 > $O/bench.json 2> $O/bench.err \
  || { tail -n 30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench',d['ms_per_step'],d['roofline']['gram_ms'],d['roofline']['frac'])"
