#!/bin/bash
# round 5: column passes in isolation (tools/bench_cols.py) and their wave-state / texture counters,
# beside the read-pattern microbenchmark's (tools/micro/colread)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python -u tools/bench_cols.py --reps 10 > $O/bench_cols.json 2> $O/bench_cols.err || { tail -n 20 $O/bench_cols.err; exit 1; }
cat $O/bench_cols.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/p1 -- python3 $R/tools/bench_cols.py --reps 2 > $O/p1.log 2>&1 || { tail -n 20 $O/p1.log; exit 1; }
echo p1 ok
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc TA_TA_BUSY TD_TD_BUSY TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE -d $O/p2 -- python3 $R/tools/bench_cols.py --reps 2 > $O/p2.log 2>&1 || { tail -n 20 $O/p2.log; exit 1; }
echo p2 ok
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/p3 -- $R/tools/micro/colread > $O/p3.log 2>&1 || { tail -n 20 $O/p3.log; exit 1; }
echo p3 ok
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc TA_TA_BUSY TD_TD_BUSY TCP_PENDING_STALL_CYCLES GRBM_GUI_ACTIVE -d $O/p4 -- $R/tools/micro/colread > $O/p4.log 2>&1 || { tail -n 20 $O/p4.log; exit 1; }
echo p4 ok
