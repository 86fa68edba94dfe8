#!/bin/bash
# round 3: the collective path (torch.distributed + RCCL) at world 1, 1/8-bins shape and config 2:
# step time against the plain path, plus a kernel/copy timeline of the 1/8-bins run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r03aa
mkdir -p $O
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 GRID_BENCH_FORCE_DIST=1
B="--steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0"
timeout -k 10 200 python -u bench.py --bins 375000 $B > $O/dist_bins375k.json 2> $O/dist.err &&
timeout -k 10 200 python -u bench.py $B > $O/dist_config2.json 2>> $O/dist.err &&
GRID_BENCH_FORCE_DIST=0 timeout -k 10 200 python -u bench.py --bins 375000 $B > $O/plain_bins375k.json 2>> $O/dist.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --bins 375000 --steps 5 --warmup 2 --no-cpu-baseline --config3-steps 0 > $O/trace.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03aa/*.json")):
    d = json.load(open(f)); s = d.get("stages_ms", {})
    print(f.split("/")[-1], round(d["ms_per_step"], 3), s)
PY
exit $rc
