#!/bin/bash
# round 4: the int32 row-block kernel's plain-block finish (GRID_ROWBLK16_XOR also selects it) -- bits with
# the product library and with the knob live, then timing on the int32 depth form at config 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_depth16.py tests/test_gpu_kernels.py tests/test_gpu_scale.py tests/test_gpu_streamed.py \
  > $O/pytest_product.log 2>&1 || { tail -n 40 $O/pytest_product.log; exit 1; }
tail -n 1 $O/pytest_product.log
GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so timeout -k 10 300 python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_depth16.py > $O/pytest_depth16_probes.log 2>&1 \
  || { tail -n 40 $O/pytest_depth16_probes.log; exit 1; }
tail -n 1 $O/pytest_depth16_probes.log
for x in 0 1 0 1; do
  GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so GRID_ROWBLK16_XOR=$x timeout -k 10 200 python -u bench.py \
    --depth-format int32 --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0 --no-files-config2 \
    > $O/rb32_xor$x.json 2> $O/rb32_xor$x.err || { tail -n 20 $O/rb32_xor$x.err; exit 1; }
  python -c "import json; d=json.load(open('$O/rb32_xor$x.json')); print('int32 xor', $x, round(d['ms_per_step'],3), d['stages_ms']['row_means'])"
done
# the 1/8-bins per-rank step's kernel timeline (where the time between the stages goes)
(cd /tmp && export TMPDIR=/tmp &&
 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace375 -- python3 \
   $GRAFT_REPO_ROOT/bench.py --bins 375000 --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0 \
   --no-files-config2 > $GRAFT_REPO_ROOT/$O/trace375.log 2>&1) || { tail -n 20 $O/trace375.log; exit 1; }
python tools/trace_step.py $(ls $O/trace375/*/*_kernel_trace.csv | head -n 1) > $O/timeline375.txt
tail -n 1 $O/timeline375.txt
