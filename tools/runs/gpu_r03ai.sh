#!/bin/bash
# round 3: full GPU-box pass 16x16x32 Gram default + copy-stream ordering (grid_stream_after) -- every -m gpu test (the long configs too),
# smoke, the default bench line, rocprofv3 kernel stats and the FETCH/WRITE PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r03ai
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 && echo "pytest: $(tail -n 1 $O/pytest_gpu.log)" &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" &&
cd /tmp && export TMPDIR=/tmp &&
B="$GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --config3-steps 0" &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 $B > $O/stats.log 2>&1 && echo "stats ok" &&
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/pmc_fetch -- python3 $B > $O/pmc_fetch.log 2>&1 && echo "pmc fetch ok" &&
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/pmc_write -- python3 $B > $O/pmc_write.log 2>&1 && echo "pmc write ok"
rc=$?
cat $O/bench.json
exit $rc
