#!/bin/bash
# round 3: host-planned row-tail kernel (tests at every tail length class), device-resident
# selection (pass C) and deferred zquant/dipCN status reads (chain tests), then the column
# statistics at the 1/8-bins shape under the probes build's column-kernel variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_depth16.py tests/test_gpu_kernels.py tests/test_gpu_sharded.py tests/test_gpu_streamed.py \
  tests/test_gpu_zq16.py tests/test_gpu_scale.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 &&
timeout -k 10 120 python -u bench.py --bins 375000 --steps 20 --warmup 3 --no-cpu-baseline --config3-steps 0 > $O/bins375k.json 2> $O/bins375k.err &&
P=$GRAFT_REPO_ROOT/grid_amd/_lib/libgridhip_probes.so
B="bench.py --bins 375000 --steps 20 --warmup 3 --no-cpu-baseline --config3-steps 0"
for v in "X=0" "GRID_COL_CU=16" "GRID_COL_PF=1" "GRID_COL16_VW=1" "GRID_COL16_VW=4" "GRID_COL_CU=16 GRID_COL_NT=0"; do
  env GRID_AMD_LIB=$P $v timeout -k 10 120 python -u $B > $O/v_${v// /_}.json 2>> $O/variants.err || exit 1
done
rc=$?
tail -n 3 $O/pytest.log
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03t/*.json")):
    d = json.load(open(f)); s = d.get("stages_ms", {})
    print(f.split("/")[-1], d["ms_per_step"], {k: s.get(k) for k in ("row_means", "col_stats", "select_sort", "zquant_gram")})
PY
exit $rc
