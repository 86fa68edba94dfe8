#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke(), the default bench line.
# Each step has its own time limit; a timeout or crash (124/137/134/139)
# ends the call, an ordinary test failure does not stop the bench.
#   bash tools/gpu_pass.sh TAG [pytest-args...]
TAG=${1:-r02}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
fatal() { case $1 in 124|137|134|139) echo "FATAL rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $O/pytest_gpu.log)"; fatal $rc pytest
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 $O/smoke.log)"; fatal $rc smoke
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; fatal $rc bench
