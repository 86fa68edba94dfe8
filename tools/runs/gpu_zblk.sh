#!/bin/bash
# Timing probe (tools build): k_zquant7 with the step-4 output blocked by 1024 columns
# (each workgroup's 8 x 1024 codes contiguous) vs row-major rows 5.4 MB apart.
set -e
O=gpurun_out/zblk; mkdir -p $O
timeout -k 10 300 python -u tools/bench_zquant.py --q16 --reps 3 --ldz-align 1024 --env "GRID_Z7_ZBLK=0;GRID_Z7_ZBLK=1;GRID_Z7_ZBLK=1,GRID_Z7_PROBE=2;GRID_Z7_ZBLK=0,GRID_Z7_PROBE=2" > $O/zq.log 2>&1
cat $O/zq.log
