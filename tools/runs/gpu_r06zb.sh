#!/bin/bash
# round 6: the bench line's ingest_roofline leg (live HIP-event timing of the ingest's inflate launch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zb
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --steps 2 --warmup 1 --config3-steps 0 --no-cpu-baseline \
  > $O/bench.json 2> $O/bench.err || { tail -n 30 $O/bench.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(round(d['ms_per_step']), d['value']);print(json.dumps(d['ingest_roofline']))"
grep "inflate leg" $O/bench.err || true
