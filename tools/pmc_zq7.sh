#!/bin/bash
# k_zquant7 wave-state counters (tools/bench_zquant.py --q16) and the gfx950 counter list.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmczq7
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD -d $O/p1 -- python3 $R/tools/bench_zquant.py --q16 --reps 1 > $O/p1.log 2>&1
echo p1 ok
