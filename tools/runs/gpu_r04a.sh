#!/bin/bash
# round 4: the copy-stream -> kernel coherence probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 120 ./tools/micro/xstream 30 > $O/xstream.jsonl 2>&1
rc=$?
cat $O/xstream.jsonl
exit $rc
