#!/bin/bash
# round 4, final tree: the default bench line (with from-files config 2 and the CPU baselines), then the
# rocprofv3 kernel statistics of the same workload
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r04q
mkdir -p $O
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err && echo "bench ok" &&
(cd /tmp && export TMPDIR=/tmp &&
 timeout -k 10 250 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 $GRAFT_REPO_ROOT/bench.py \
   --steps 3 --warmup 1 --no-cpu-baseline --config3-steps 0 --no-files-config2 > $O/stats.log 2>&1) && echo "stats ok"
rc=$?
head -c 900 $O/bench.json; echo
exit $rc
