#!/bin/bash
# round 6: the distributed drop-in on the GPU (ranks sharing it under gloo), the single-GPU drop-in after the
# writer refactor, then a short bench with the from-files headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dist_wgs.py tests/test_gpu_e2e.py tests/test_gpu_gzwrite.py tests/test_gpu_cohort.py > $O/pytest.log 2>&1 \
  || { tail -n 60 $O/pytest.log; exit 1; }
tail -n 3 $O/pytest.log
timeout -k 10 480 python -u bench.py --steps 2 --warmup 1 --config3-steps 0 --no-cpu-baseline \
  > $O/bench.json 2> $O/bench.err || { tail -n 40 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('value', d['value'], d['ms_per_step'], d.get('from_files',{}).get('stages_s'), d['device_chain']['ms_per_step'])"
