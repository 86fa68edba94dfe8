#!/bin/bash
# round 4: host read rate and host -> HBM copy rate from pinned vs pageable staging
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 200 python -u tools/e2e_files.py --bgzf --generate-only --samples 400 > $O/gen.log 2>&1 || { tail -n 20 $O/gen.log; exit 1; }
timeout -k 10 200 python -u tools/bench_read.py /dev/shm/grid_e2e/mosdepth --gb 4 > $O/read.jsonl 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e
cat $O/read.jsonl
exit $rc
