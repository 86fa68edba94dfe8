#!/bin/bash
# round 5: kernel statistics of the from-files config-2 run after the inflate rework (threads 1): where the ingest's
# device time goes now (inflate vs the mosdepth parse)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r05an
mkdir -p $O
export TMPDIR=/tmp
D=/dev/shm/grid_r05an
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --generate-only --reuse > $O/gen.log 2>&1 \
  || { tail -n 20 $O/gen.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 tools/e2e_files.py --bgzf \
  --data $D --reuse --threads 1 --json $O/e2e_t1_prof.json > $O/e2e.log 2>&1 || { tail -n 30 $O/e2e.log; rm -rf $D; exit 1; }
rm -rf $D
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/kernel_stats.csv')))[:14]:
  print(r['Name'][:50], r['Calls'], round(float(r['TotalDurationNs'])/1e9,3), 's', r['Percentage'])
"
