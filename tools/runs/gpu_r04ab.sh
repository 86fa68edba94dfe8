#!/bin/bash
# round 4: k_zquant7 loads the upper 16 B of a lane's code window only when its columns reach past the first
# 8 codes -- the step-4 parity tests (product library), then the A/B against always loading it
# (GRID_Z7_HIALL=1, tools build) at config 2 and at the 1/8-bins shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_depth16.py tests/test_gpu_zq16.py tests/test_gpu_kernels.py tests/test_gpu_scale.py \
  tests/test_gpu_e2e.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for bins in 3000000 375000; do
  for h in 1 0 1 0; do
    GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so GRID_Z7_HIALL=$h timeout -k 10 200 python -u bench.py \
      --bins $bins --steps 10 --warmup 2 --no-cpu-baseline --config3-steps 0 --no-files-config2 \
      > $O/z7_b${bins}_hiall$h.json 2> $O/z7_b${bins}_hiall$h.err || { tail -n 20 $O/z7_b${bins}_hiall$h.err; exit 1; }
    python -c "import json; d=json.load(open('$O/z7_b${bins}_hiall$h.json')); print('bins $bins hiall $h', round(d['ms_per_step'],3), d['stages_ms']['zquant_gram'], round(d['roofline']['gram_ms'],3))"
  done
done
