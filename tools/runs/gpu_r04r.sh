#!/bin/bash
# round 4: the row-block kernel's plain-block sums by lane exchanges (GRID_ROWBLK16_XOR, default 1) and the
# streamed form (GRID_ROWBLK16_PB=0) -- bits with the knobs live (tools build) and with the product library,
# then timing at config 2 and at the 1/8-bins per-rank shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04r
mkdir -p $O
GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_depth16.py > $O/pytest_depth16_probes.log 2>&1 \
  || { tail -n 40 $O/pytest_depth16_probes.log; exit 1; }
tail -n 1 $O/pytest_depth16_probes.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_depth16.py tests/test_gpu_kernels.py tests/test_gpu_scale.py > $O/pytest_product.log 2>&1 \
  || { tail -n 40 $O/pytest_product.log; exit 1; }
tail -n 1 $O/pytest_product.log
for bins in 375000 3000000; do
  for c in "1 0" "1 1" "0 1" "1 0" "1 1"; do
    set -- $c
    tag=b${bins}_pb$1_xor$2
    GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so GRID_ROWBLK16_PB=$1 GRID_ROWBLK16_XOR=$2 \
      timeout -k 10 200 python -u bench.py --bins $bins --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0 \
      --no-files-config2 > $O/rb_$tag.json 2> $O/rb_$tag.err || { tail -n 20 $O/rb_$tag.err; exit 1; }
    python -c "import json; d=json.load(open('$O/rb_$tag.json')); print('$tag', round(d['ms_per_step'],3), d['stages_ms']['row_means'])"
  done
done
