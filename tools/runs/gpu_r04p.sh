#!/bin/bash
# round 4, final tree: every -m gpu test and smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r04p
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 && echo "pytest: $(tail -n 1 $O/pytest_gpu.log)" &&
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok"
rc=$?
grep -E "passed|failed|error" $O/pytest_gpu.log | tail -n 3
exit $rc
