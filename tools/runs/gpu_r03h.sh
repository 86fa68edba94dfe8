#!/bin/bash
# round 3: from-files config 2 (BGZF mosdepth cohort in /dev/shm): device ingest vs host
# parser, both with the step-4 -> step-5 hand-off; output-disk write rate
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03h
mkdir -p $O
(df -h /tmp /dev/shm; nproc; free -g) > $O/box.txt 2>&1
(timeout -k 10 120 dd if=/dev/zero of=/tmp/grid_dd_test bs=1M count=8192 conv=fdatasync 2>&1; rm -f /tmp/grid_dd_test) >> $O/box.txt
timeout -k 10 900 python -u tools/e2e_files.py --bgzf --device-ingest --reuse --json $O/e2e_dev.json > $O/e2e_dev.log 2>&1 &&
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --reuse --json $O/e2e_host.json > $O/e2e_host.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
cat $O/box.txt; tail -n 25 $O/e2e_dev.log; tail -n 20 $O/e2e_host.log
exit $rc
