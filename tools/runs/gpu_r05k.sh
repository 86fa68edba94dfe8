#!/bin/bash
# round 5: kernel timeline of the from-files config-2 ingest at threads 16 (rocprofv3 kernel trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05k
mkdir -p $O
D=/dev/shm/grid_r05k
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --generate-only --reuse > $O/gen.log 2>&1 \
  || { tail -n 20 $O/gen.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
GRID_INGEST_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -- \
  python3 $R/tools/e2e_files.py --bgzf --data $D --reuse --threads 16 --json $O/e2e_t16.json > $O/e2e_t16.log 2>&1 \
  || { tail -n 30 $O/e2e_t16.log; rm -rf $D; exit 1; }
rm -rf $D
ls $O/trace/*/
