set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g7b
timeout -k 10 300 python -u tools/bench_gram.py --variants 6,7,8,14,15 --reps 2 > gpurun_out/g7b/b.log 2>&1
cat gpurun_out/g7b/b.log | grep min
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P="python3 $R/tools/bench_gram.py --variants 6,7 --reps 1"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $R/gpurun_out/g7b/pmc2 -- $P > $R/gpurun_out/g7b/pmc2.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/g7b/pmc3 -- $P > $R/gpurun_out/g7b/pmc3.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $R/gpurun_out/g7b/pmc1 -- $P > $R/gpurun_out/g7b/pmc1.log 2>&1
echo done
