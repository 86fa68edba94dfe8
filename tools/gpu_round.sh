#!/bin/bash
# Full GPU-box pass for one round tag: GPU parity tests, smoke(), the default
# bench line, rocprofv3 kernel stats of the same bench command, and the two
# HBM-traffic PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass).
#   bash tools/gpu_round.sh TAG [skip-tests]
# Output: gpurun_out/TAG/{pytest_gpu.log,smoke.log,bench.json,stats/,pmc_fetch/,pmc_write/}
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  echo "pytest ok: $(tail -1 $O/pytest_gpu.log)"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  echo "smoke ok"
fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
echo "bench ok"; cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --config3-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 $B > $O/stats.log 2>&1
echo "stats ok"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/pmc_fetch -- python3 $B > $O/pmc_fetch.log 2>&1
echo "pmc fetch ok"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/pmc_write -- python3 $B > $O/pmc_write.log 2>&1
echo "pmc write ok"
