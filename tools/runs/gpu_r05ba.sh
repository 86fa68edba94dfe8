#!/bin/bash
# round 5: PMC read of the production Gram (k_gram8, LAY 4) at config 2 on random data (tools/bench_gram.py):
# texture-path busy (the L2 -> LDS feed), MFMA busy, GPU clock
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ba
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc TA_TA_BUSY TD_TD_BUSY TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE \
  -d $O/p1 -- python3 $R/tools/bench_gram.py --reps 2 --variants kb21 > $O/p1.log 2>&1 || { tail -n 20 $O/p1.log; exit 1; }
echo p1 ok
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_COUNT \
  -d $O/p2 -- python3 $R/tools/bench_gram.py --reps 2 --variants kb21 > $O/p2.log 2>&1 || { tail -n 20 $O/p2.log; exit 1; }
echo p2 ok
