#!/bin/bash
# round 3, final tree: every -m gpu test, smoke, the default bench line, rocprofv3 kernel stats, then the
# GPU inflate (2^8 fast table, 28 waves per CU) on 1,024 BGZF files and from-files config 2 (BGZF)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r03ap
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 && echo "pytest: $(tail -n 1 $O/pytest_gpu.log)" &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo "smoke ok" &&
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" &&
(cd /tmp && export TMPDIR=/tmp &&
 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --config3-steps 0 > $O/stats.log 2>&1) && echo "stats ok" &&
GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/bench_dev_ingest.py --samples 1024 --modes gpu --json $O/dev_ingest_1024.json > $O/dev_ingest.log 2>&1 &&
rm -rf /dev/shm/grid_dev_ingest &&
GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/e2e_files.py --bgzf --json $O/e2e_bgzf.json > $O/e2e_bgzf.log 2>&1
rc=$?
rm -rf /dev/shm/grid_dev_ingest /dev/shm/grid_e2e /tmp/grid_e2e_out
tail -n 2 $O/pytest_gpu.log; cat $O/bench.json | head -c 600; echo
grep -v "batch files" $O/dev_ingest.log | grep -v generated | tail -n 4
grep "e2e\]" $O/e2e_bgzf.log | grep -v " files$" | tail -n 12
exit $rc
