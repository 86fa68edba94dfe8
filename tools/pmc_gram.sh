# PMC passes over the Gram microbenchmark (one variant): SQ issue/wait mix,
# LDS conflicts, TA/TD busy.  VARS=kb21 bash tools/pmc_gram.sh
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcg
mkdir -p $O
P="python3 $R/tools/bench_gram.py --variants ${VARS:-kb21} --reps 1"
timeout -s KILL 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $O/p1 -- $P > $O/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC -d $O/p2 -- $P > $O/p2.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum -d $O/p3 -- $P > $O/p3.log 2>&1 || echo "p3 failed"
echo done
