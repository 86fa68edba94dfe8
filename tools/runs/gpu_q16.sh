#!/bin/bash
# Compact-depth (q16) pass: its GPU tests, the bench line, a knob sweep and kernel stats.
#   bash tools/gpu_q16.sh TAG
set -e
TAG=${1:-q16}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_q16.log 2>&1
echo "pytest ok: $(tail -1 $O/pytest_q16.log)"
B="bench.py --depth-format q16 --no-cpu-baseline --steps 5 --warmup 1"
timeout -k 10 200 python -u $B > $O/bench_q16.json 2> $O/bench_q16.err
cat $O/bench_q16.json
for kv in "GRID_COL16_VW=1" "GRID_COL16_CU=16" "GRID_ROWBLK16_PB=2"; do
  env $kv timeout -k 10 200 python -u $B > $O/bench_q16_$kv.json 2>> $O/bench_q16.err
  echo "$kv $(python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['ms_per_step'],d['stages_ms'])" $O/bench_q16_$kv.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_q16 -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --depth-format q16 > $O/stats_q16.log 2>&1
echo "stats ok"
