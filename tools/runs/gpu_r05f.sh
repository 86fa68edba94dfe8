#!/bin/bash
# round 5: column-pass read-pattern microbenchmark (tools/micro/colread.hip)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 120 tools/micro/colread > $O/colread.jsonl 2>&1 || { cat $O/colread.jsonl; exit 1; }
cat $O/colread.jsonl
