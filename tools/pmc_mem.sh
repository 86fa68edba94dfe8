#!/bin/bash
# Memory-side stall counters for k_zquant7 (tools/bench_zquant.py --q16) and k_gram8 (tools/bench_gram.py):
# one rocprofv3 --pmc pass per counter group (<= 4 TCC, 2 TA, 2 TD, 2 GRBM per pass).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmcmem
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ZQ="python3 $R/tools/bench_zquant.py --q16 --reps 1"
GR="python3 $R/tools/bench_gram.py --reps 1 --variants kb21"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc TCC_EA0_WRREQ_STALL TCC_TOO_MANY_EA_WRREQS_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL GRBM_GUI_ACTIVE -d $O/zq1 -- $ZQ > $O/zq1.log 2>&1
echo zq1 ok
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_TAG_STALL TCC_BUSY GRBM_GUI_ACTIVE -d $O/zq2 -- $ZQ > $O/zq2.log 2>&1
echo zq2 ok
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc TA_TA_BUSY TD_TD_BUSY TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE -d $O/zq3 -- $ZQ > $O/zq3.log 2>&1
echo zq3 ok
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_TAG_STALL TCC_BUSY GRBM_GUI_ACTIVE -d $O/gr2 -- $GR > $O/gr2.log 2>&1
echo gr2 ok
