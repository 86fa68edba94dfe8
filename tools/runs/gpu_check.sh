#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke(), bench line, rocprofv3 kernel stats.
#   bash tools/gpu_check.sh TAG
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest ok"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench ok"; cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/stats.log 2>&1
echo "stats ok"
