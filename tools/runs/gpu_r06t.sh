#!/bin/bash
# round 6: k_md_parse at 8 waves per SIMD with 3 loads in flight (grid_amd/_lib) against 5 / 6
# (grid_amd/_lib_mdref), and the per-file chunk scan as a workgroup scan: from-files bench (K = 3) alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_ingest.py tests/test_gpu_e2e.py tests/test_gpu_dist_wgs.py \
  > $O/pytest.log 2>&1 || { tail -n 60 $O/pytest.log; exit 1; }
echo "new: $(tail -n 1 $O/pytest.log)"
for v in new ref ref2 new2; do
  lib=grid_amd/_lib/libgridhip.so; [ ${v%2} = ref ] && lib=grid_amd/_lib_mdref/libgridhip.so
  GRID_AMD_LIB=$lib timeout -k 10 500 python3 bench.py --steps 3 --warmup 1 --config3-steps 0 --no-cpu-baseline \
    --keep-files > $O/bench_$v.json 2> $O/bench_$v.err || { tail -n 30 $O/bench_$v.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', round(d['ms_per_step']), d['from_files']['stages_s'], 'chain', round(d['device_chain']['ms_per_step'],2))"
done
rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out
