#!/bin/bash
# round 3: kernel timeline of the 1/8-bins shape after the row-tail kernel, device-resident
# selection and deferred status reads (r03s was before them)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r03v
mkdir -p $O
timeout -k 10 120 python -u bench.py --bins 375000 --steps 20 --warmup 3 --no-cpu-baseline --config3-steps 0 > $O/bench_bins375k.json 2> $O/bench_bins375k.err &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --bins 375000 --steps 5 --warmup 2 --no-cpu-baseline --config3-steps 0 > $O/trace.log 2>&1
rc=$?
cat $O/bench_bins375k.json
find $O/trace -name "*.csv" | head
exit $rc
