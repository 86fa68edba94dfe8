#!/bin/bash
# round 5, first call: the round-4 tree's default bench line (device chain only) and its kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-files-baseline \
  --no-files-config2 --config3-steps 0 > $O/bench.json 2> $O/bench.err || { tail -n 30 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-files-baseline --no-files-config2 \
  --config3-steps 0 > $GRAFT_REPO_ROOT/$O/stats.log 2>&1 || { tail -n 30 $GRAFT_REPO_ROOT/$O/stats.log; exit 1; }
echo stats ok
