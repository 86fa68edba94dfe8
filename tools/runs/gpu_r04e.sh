#!/bin/bash
# round 4: host read rate of the BGZF cohort (tools/bench_read.py), then from-files config 2 again
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04e
mkdir -p $O
GRID_INGEST_TRACE=1 timeout -k 10 600 python -u tools/e2e_files.py --bgzf --reuse --json $O/e2e_files_config2_bgzf.json \
  > $O/e2e.log 2>&1 || { tail -n 30 $O/e2e.log; exit 1; }
grep -E "ingest\]|e2e\]" $O/e2e.log | tail -n 14
timeout -k 10 300 python -u tools/bench_read.py /dev/shm/grid_e2e/mosdepth --gb 8 > $O/read.jsonl 2>&1
rc=$?
cat $O/read.jsonl
rm -rf /dev/shm/grid_e2e
exit $rc
