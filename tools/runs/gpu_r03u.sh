#!/bin/bash
# round 3: column-kernel variants at the 1/8-bins shape (probes build), after r03t
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 120 python -u bench.py --bins 375000 --steps 20 --warmup 3 --no-cpu-baseline --config3-steps 0 > $O/bins375k.json 2> $O/bins375k.err &&
P=$GRAFT_REPO_ROOT/grid_amd/_lib/libgridhip_probes.so
B="bench.py --bins 375000 --steps 20 --warmup 3 --no-cpu-baseline --config3-steps 0"
for v in "X=0" "GRID_COL_CU=16" "GRID_COL_PF=1" "GRID_COL16_VW=1" "GRID_COL16_VW=4" "GRID_COL_CU=16 GRID_COL_NT=0"; do
  env GRID_AMD_LIB=$P $v timeout -k 10 120 python -u $B > $O/v_${v// /_}.json 2>> $O/variants.err || exit 1
done
rc=$?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03u/*.json")):
    d = json.load(open(f)); s = d.get("stages_ms", {})
    print(f.split("/")[-1], d["ms_per_step"], {k: s.get(k) for k in ("row_means", "col_stats", "select_sort", "zquant_gram")})
PY
exit $rc
