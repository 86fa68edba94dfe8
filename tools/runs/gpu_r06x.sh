#!/bin/bash
# round 6: is the pipelined ingest bound by the host's read + copy of each 4 GB batch? per-batch phase
# times (GRID_INGEST_TRACE) with 8 (default) and 16 file-read threads, from-files K = 2 on one cohort
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06x
mkdir -p $O
export TMPDIR=/tmp
for v in rt8 rt16 rt8b rt16b; do
  rt=${v#rt}; rt=${rt%b}
  GRID_INGEST_TRACE=1 GRID_INGEST_READ_THREADS=$rt timeout -k 10 500 python3 bench.py --steps 2 --warmup 1 \
    --config3-steps 0 --no-cpu-baseline --keep-files > $O/bench_$v.json 2> $O/bench_$v.err \
    || { tail -n 30 $O/bench_$v.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', round(d['ms_per_step']), d['from_files']['stages_s'])"
done
rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out
grep -m 40 "\[ingest\]" $O/bench_rt8b.err | tail -20
