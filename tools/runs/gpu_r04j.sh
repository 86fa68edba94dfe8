#!/bin/bash
# round 4: pageable ingest staging -- ingest GPU tests, then the driver's bench command (N=1, with the
# from-files config-2 record)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
GRID_INGEST_TRACE=1 timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?
tail -n 5 $O/bench.err
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); f=d.get('from_files_config2',{})
print('value', d['value'], 'ms/step', d['ms_per_step']); print('from files', {k: f.get(k) for k in ('value','steps_4_7_s','stages_s','cohort_generation_s','skipped')})"
exit $rc
