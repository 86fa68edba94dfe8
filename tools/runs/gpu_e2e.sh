#!/bin/bash
# The from-files end-to-end run at config 2 (tools/e2e_files.py): per-step wall
# times of the drop-in steps 4-7 and peak host RSS.   bash tools/gpu_e2e.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-e2e}
mkdir -p $O
cd $R
timeout -k 10 1100 python -u tools/e2e_files.py --json $O/e2e_files.json 2> $O/e2e_files.err > $O/e2e_files.out
rc=$?; echo "e2e rc=$rc"; tail -3 $O/e2e_files.err; exit $rc
