#!/bin/bash
# k_zquant7 grid walk (super-tiles) and step-4 output row alignment A/B; zquant GPU tests
set -e
O=gpurun_out/zq7; mkdir -p $O
E="GRID_Z7_RGS=0;GRID_Z7_RGS=8,GRID_Z7_CBW=64;GRID_Z7_RGS=16,GRID_Z7_CBW=64;GRID_Z7_RGS=32,GRID_Z7_CBW=32;GRID_Z7_RGS=4,GRID_Z7_CBW=128;GRID_Z7_RGS=2,GRID_Z7_CBW=512;GRID_Z7_RGS=16,GRID_Z7_CBW=64,GRID_Z7_PROBE=1;GRID_Z7_RGS=16,GRID_Z7_CBW=64,GRID_Z7_PROBE=2"
timeout -k 10 300 python -u tools/bench_zquant.py --q16 --reps 3 --env "$E" > $O/zq8.log 2>&1
cat $O/zq8.log
timeout -k 10 300 python -u tools/bench_zquant.py --q16 --reps 3 --ldz-align 64 --env "GRID_Z7_RGS=0;GRID_Z7_RGS=16,GRID_Z7_CBW=64;GRID_Z7_RGS=0,GRID_Z7_PROBE=2" > $O/zq64.log 2>&1
cat $O/zq64.log
