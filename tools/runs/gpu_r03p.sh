#!/bin/bash
# round 3: from-files config 2 (BGZF) with the 8 KiB inflate ring and the re-seeded split;
# then the full pass (tools/runs/gpu_r03n.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03p
mkdir -p $O
GRID_INGEST_TRACE=1 timeout -k 10 500 python -u tools/e2e_files.py --bgzf --json $O/e2e_bgzf.json > $O/e2e_bgzf.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
grep "e2e\]" $O/e2e_bgzf.log | grep -v " files$" | tail -n 16; grep "batches done\|gathered" $O/e2e_bgzf.log
[ $rc -eq 0 ] && bash tools/runs/gpu_r03n.sh
