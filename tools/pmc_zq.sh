#!/bin/bash
# zquant timing and PMC counters (tools/bench_zquant.py, q16 source).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmczq
mkdir -p $O
E="GRID_ZQUANT_NT=1;GRID_ZQUANT7=0"
timeout -k 10 200 python3 $R/tools/bench_zquant.py --q16 --reps 3 --env "$E" > $O/t.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $O/p3 -- python3 $R/tools/bench_zquant.py --q16 --reps 1 --env "$E" > $O/p3.log 2>&1
echo p3 ok
