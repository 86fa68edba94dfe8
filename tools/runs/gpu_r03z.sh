#!/bin/bash
# round 3: row means one wave per row (k_row_means), the kth passes restored -- tests, then
# the 1/8-bins shape and config 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_depth16.py tests/test_gpu_sharded.py tests/test_gpu_streamed.py \
  tests/test_gpu_zq16.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -u bench.py --bins 375000 --steps 20 --warmup 3 --no-cpu-baseline --config3-steps 0 > $O/bins375k.json 2> $O/bench.err &&
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0 > $O/config2.json 2>> $O/bench.err
rc=$?
tail -n 3 $O/pytest.log
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03z/*.json")):
    d = json.load(open(f)); s = d.get("stages_ms", {})
    print(f.split("/")[-1], round(d["ms_per_step"], 3), s)
PY
exit $rc
