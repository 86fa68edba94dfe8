#!/bin/bash
# round 6: k_md_parse with the reference line's K index and key loaded before the line is parsed
# (grid_amd/_lib) against the parse of e6c7b3a (grid_amd/_lib_mdref): from-files bench (K = 3) alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_ingest.py tests/test_gpu_e2e.py tests/test_gpu_dist_wgs.py \
  > $O/pytest.log 2>&1 || { tail -n 60 $O/pytest.log; exit 1; }
echo "pf: $(tail -n 1 $O/pytest.log)"
for v in pf ref ref2 pf2; do
  lib=grid_amd/_lib/libgridhip.so; [ ${v%2} = ref ] && lib=grid_amd/_lib_mdref/libgridhip.so
  GRID_AMD_LIB=$lib timeout -k 10 500 python3 bench.py --steps 3 --warmup 1 --config3-steps 0 --no-cpu-baseline \
    --keep-files > $O/bench_$v.json 2> $O/bench_$v.err || { tail -n 30 $O/bench_$v.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', round(d['ms_per_step']), d['from_files']['stages_s'], 'chain', round(d['device_chain']['ms_per_step'],2))"
done
# the device writer's pwrite threads per batch (probes build: GRID_WRITER_W), same cohort
for w in 4 8; do
  GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so GRID_WRITER_W=$w timeout -k 10 500 python3 bench.py --steps 3 --warmup 1 \
    --config3-steps 0 --no-cpu-baseline --keep-files > $O/bench_w$w.json 2> $O/bench_w$w.err \
    || { tail -n 30 $O/bench_w$w.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_w$w.json'));print('W$w', round(d['ms_per_step']), d['from_files']['stages_s'])"
done
rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out
