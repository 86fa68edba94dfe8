#!/bin/bash
# Configs 3 and 4 on one GPU (bin-streamed): rocprofv3 kernel stats of one
# config-3 step, PMC traffic passes of the default (config 2) bench, and a
# config-4 bench line.  Each step has its own time limit; the script stops
# at the first failure.
#   bash tools/gpu_cfg34.sh TAG [skip-cfg4]
set -e
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B3="$R/bench.py --samples 50000 --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats3 -- python3 $B3 > $O/stats3.log 2>&1
echo "config-3 stats ok"
B2="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats2 -- python3 $B2 > $O/stats2.log 2>&1
echo "config-2 stats ok"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/pmc_fetch -- python3 $B2 > $O/pmc_fetch.log 2>&1
echo "pmc fetch ok"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/pmc_write -- python3 $B2 > $O/pmc_write.log 2>&1
echo "pmc write ok"
if [ "$2" != "skip-cfg4" ]; then
  cd $R
  timeout -k 10 600 python3 -u bench.py --samples 50000 --bins 30000000 --steps 1 --warmup 1 --cpu-samples 2048 \
    > $O/bench_cfg4.json 2> $O/bench_cfg4.err
  echo "config-4 bench ok"; cat $O/bench_cfg4.json
fi
