#!/bin/bash
# round 4: kernel stats of the from-files config-2 steps (cohort written first, outside the profiler)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04g
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --generate-only > $O/gen.log 2>&1 || { tail -n 20 $O/gen.log; exit 1; }
GRID_INGEST_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- \
  python3 -u tools/e2e_files.py --bgzf --reuse --json $O/e2e.json > $O/e2e.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e
grep -E "e2e\] .*(step4_ingest|step4_write|done in)" $O/e2e.log | tail -n 8
find $O/stats -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
head -n 25 $O/kernel_stats.csv | cut -c1-220
find $O/stats -name "*kernel_trace.csv" -exec gzip -c {} \; > $O/kernel_trace.csv.gz
exit $rc
