#!/bin/bash
# The from-files end-to-end run at config 2 (drop-in steps 4-7 on a generated 3,202 x 3M mosdepth
# cohort) on the current tree.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02aj
mkdir -p $O
cd $R
timeout -k 10 1000 python -u tools/e2e_files.py --json $O/e2e_files.json 2> $O/e2e_files.err > $O/e2e_files.out
rc=$?; echo "e2e rc=$rc"; tail -3 $O/e2e_files.err; [ $rc -eq 0 ] || exit $rc
cat $O/e2e_files.json
