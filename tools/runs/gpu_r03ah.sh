#!/bin/bash
# round 3: control arm of r03ag (device ingest without the copy-stream ordering), once
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ah
mkdir -p $O
timeout -k 10 200 python -u tools/runs/xstream_probe.py > $O/control_no_wait.log 2>&1
rc=$?
echo "control arm (no wait) rc=$rc"; tail -n 30 $O/control_no_wait.log
exit 0
