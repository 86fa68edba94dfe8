#!/bin/bash
# round 3: pipelined compact column statistics (k_col16_pipe) -- q16 == int32 tests, then the
# 1/8-bins shape and config 2 with the new kernel and with GRID_COL_PIPE=0 (probes build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_depth16.py tests/test_gpu_kernels.py > $O/pytest.log 2>&1 &&
P=$GRAFT_REPO_ROOT/grid_amd/_lib/libgridhip_probes.so &&
for b in 375000 3000000; do
  timeout -k 10 200 python -u bench.py --bins $b --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0 > $O/pipe_$b.json 2>> $O/bench.err &&
  GRID_AMD_LIB=$P GRID_COL_PIPE=0 timeout -k 10 200 python -u bench.py --bins $b --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0 > $O/nopipe_$b.json 2>> $O/bench.err || exit 1
done
rc=$?
tail -n 3 $O/pytest.log
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03w/*.json")):
    d = json.load(open(f)); s = d.get("stages_ms", {})
    print(f.split("/")[-1], round(d["ms_per_step"], 3), {k: s.get(k) for k in ("row_means", "col_stats", "select_sort", "zquant_gram")})
PY
exit $rc
