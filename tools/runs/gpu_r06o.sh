#!/bin/bash
# round 6: every HIP file compiled with -structurizecfg-skip-uniform-regions (grid_amd/_lib_skipall)
# against the product build (only k_inflate's file): parity of the chain under it, then the
# from-files bench (K = 3) alternating the two libraries on one cohort
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06o
mkdir -p $O
export TMPDIR=/tmp
GRID_AMD_LIB=grid_amd/_lib_skipall/libgridhip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_e2e.py tests/test_gpu_select.py \
  > $O/pytest_skipall.log 2>&1 || { tail -n 60 $O/pytest_skipall.log; exit 1; }
echo "skipall: $(tail -n 1 $O/pytest_skipall.log)"
for v in base skipall skipall2 base2; do
  lib=grid_amd/_lib/libgridhip.so; [ ${v%2} = skipall ] && lib=grid_amd/_lib_skipall/libgridhip.so
  GRID_AMD_LIB=$lib timeout -k 10 500 python3 bench.py --steps 3 --warmup 1 --config3-steps 0 --no-cpu-baseline \
    --keep-files > $O/bench_$v.json 2> $O/bench_$v.err || { tail -n 30 $O/bench_$v.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', round(d['ms_per_step']), d['from_files']['stages_s'], 'chain', round(d['device_chain']['ms_per_step'],2))"
done
rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out
