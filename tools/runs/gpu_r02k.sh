#!/bin/bash
# GPU tests, the from-files end-to-end run at config 2, and a config-4 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $O/pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u tools/e2e_files.py --json $O/e2e_files.json 2> $O/e2e_files.err > $O/e2e_files.out
rc=$?; echo "e2e rc=$rc"; tail -3 $O/e2e_files.err; [ $rc -eq 0 ] || exit $rc
