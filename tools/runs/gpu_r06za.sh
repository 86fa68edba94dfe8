#!/bin/bash
# round 6: ingest batch ramp (1 GB, 2 GB, then 4 GB batches) -- GPU ingest tests, then
# from-files K = 2 alternating ramp / no ramp on one cohort, per-batch trace
# (the GRID_INGEST_RAMP knob this script sets was dropped with the ramp: profiles/r06za_ingest_ramp_ab.json)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06za
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_ingest.py tests/test_gpu_dist_wgs.py > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in ramp flat ramp2 flat2; do
  r="4,2"; [[ $v == flat* ]] && r=""
  GRID_INGEST_RAMP=$r GRID_INGEST_TRACE=1 timeout -k 10 500 python3 bench.py --steps 2 --warmup 1 \
    --config3-steps 0 --no-cpu-baseline --keep-files > $O/bench_$v.json 2> $O/bench_$v.err \
    || { tail -n 30 $O/bench_$v.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', round(d['ms_per_step']), d['from_files']['stages_s'], d['from_files'].get('output_digests', '')[:0] if isinstance(d['from_files'].get('output_digests'), str) else '')"
done
rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out
grep -m 30 "\[ingest\]" $O/bench_ramp2.err | tail -26
