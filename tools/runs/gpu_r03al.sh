#!/bin/bash
# round 3: RCCL path at world 1 after TorchComm.all_gather -> all_gather_into_tensor: the bench line
# (1/8-bins shape and config 2) and the sharded GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r03al
mkdir -p $O
B="--steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0"
MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 GRID_BENCH_FORCE_DIST=1 \
  timeout -k 10 200 python -u bench.py --bins 375000 $B > $O/dist_bins375k.json 2> $O/dist.err &&
MASTER_ADDR=127.0.0.1 MASTER_PORT=29562 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 GRID_BENCH_FORCE_DIST=1 \
  timeout -k 10 200 python -u bench.py $B > $O/dist_config2.json 2>> $O/dist.err &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sharded.py > $O/pytest_sharded.log 2>&1
rc=$?
tail -n 3 $O/pytest_sharded.log
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03al/*.json")):
    d = json.load(open(f)); s = d.get("stages_ms", {})
    print(f.split("/")[-1], round(d["ms_per_step"], 3), d["config"]["parallelism"], s)
PY
exit $rc
