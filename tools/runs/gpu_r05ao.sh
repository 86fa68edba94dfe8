#!/bin/bash
# round 5: where the config-3 step's non-Gram time goes (50,000 x 3 M, streamed: 7 chunks x 3 passes): stage
# breakdown of one timed step (bench --samples 50000) and its kernel statistics
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05ao
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --samples 50000 --steps 1 --warmup 1 --no-cpu-baseline --no-files-baseline --no-files-config2 --config3-steps 0"
timeout -k 10 500 python3 $B > $O/bench_cfg3.json 2> $O/bench_cfg3.err || { tail -n 20 $O/bench_cfg3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_cfg3.json'));print(d['ms_per_step'], d['stages_ms'], d['roofline']['gram_ms'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 $B > $O/prof.log 2>&1 || { tail -n 20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/kernel_stats.csv')))[:16]:
  print(r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs'])/1e6,1), 'ms', r['Percentage'])
"
