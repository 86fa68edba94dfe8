#!/bin/bash
# round 4, final tree: HBM traffic per kernel launch of the bench command (two PMC passes: FETCH_SIZE,
# WRITE_SIZE), summarised per kernel for bench.py's roofline.traffic
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04aa
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --config3-steps 0 --no-files-config2"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/pmc_fetch -- python3 $B \
  > $O/pmc_fetch.log 2>&1 && echo "pmc fetch ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/pmc_write -- python3 $B \
  > $O/pmc_write.log 2>&1 && echo "pmc write ok" &&
cd $R && python tools/pmc_traffic.py gpurun_out/r04aa gpurun_out/r04aa/pmc_traffic.json > $O/traffic.log 2>&1 &&
tail -n 12 $O/traffic.log
