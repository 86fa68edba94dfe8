set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="python3 $R/tools/bench_gram.py --variants ${VARS:-4} --reps 1"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $R/gpurun_out/pmc1 -- $P > $R/gpurun_out/pmc1.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $R/gpurun_out/pmc2 -- $P > $R/gpurun_out/pmc2.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/pmc3 -- $P > $R/gpurun_out/pmc3.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL -d $R/gpurun_out/pmc4 -- $P > $R/gpurun_out/pmc4.log 2>&1
echo done
