#!/bin/bash
# round 4: the column-statistics kernel variants -- their bits (compact-kernel parity tests with the knobs live
# in the tools build), then their timing at config 2 and at the 1/8-bins per-rank shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04o
mkdir -p $O
# the column kernel variants' bits (tools build, knobs live) before their timing
GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_depth16.py > $O/pytest_depth16_probes.log 2>&1 \
  || { tail -n 40 $O/pytest_depth16_probes.log; exit 1; }
tail -n 2 $O/pytest_depth16_probes.log
# column statistics (tools build): columns per thread (GRID_COL16_VW), raw-code software-pipelined row groups
# (GRID_COL_PF), rows per group (GRID_COL16_CU), at config 2 and at the 1/8-bins per-rank shape
for bins in 375000 3000000; do
  for c in "2 0 8" "2 1 8" "1 1 8" "1 1 16" "2 1 16"; do
    set -- $c
    tag=b${bins}_vw$1_pf$2_cu$3
    GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so GRID_COL16_VW=$1 GRID_COL_PF=$2 GRID_COL16_CU=$3 \
      timeout -k 10 200 python -u bench.py --bins $bins --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0 \
      --no-files-config2 > $O/col_$tag.json 2> $O/col_$tag.err || { tail -n 20 $O/col_$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/col_$tag.json')); print('$tag', d['ms_per_step'], d['stages_ms']['col_stats'])"
  done
done
# the Gram's flush in 512-B row segments (GRID_GRAM_WIDE): bits, then time and HBM writes at config 2
GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "gram" > $O/pytest_gram_probes.log 2>&1 \
  || { tail -n 40 $O/pytest_gram_probes.log; exit 1; }
tail -n 2 $O/pytest_gram_probes.log
for w in 0 1 0 1; do
  GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so GRID_GRAM_WIDE=$w timeout -k 10 200 python -u bench.py --steps 10 \
    --warmup 2 --no-cpu-baseline --config3-steps 0 --no-files-config2 > $O/gram_wide$w.json 2> $O/gram_wide$w.err \
    || { tail -n 20 $O/gram_wide$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/gram_wide$w.json')); print('wide', $w, d['ms_per_step'], d['roofline']['gram_ms'])"
done
export TMPDIR=/tmp
for w in 0 1; do
  GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so GRID_GRAM_WIDE=$w timeout -k 10 300 rocprofv3 --kernel-trace \
    --output-format csv --pmc WRITE_SIZE -d $O/pmc_wide$w -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    --config3-steps 0 --no-files-config2 > $O/pmc_wide$w.log 2>&1 || { tail -n 20 $O/pmc_wide$w.log; exit 1; }
done
echo pmc done
