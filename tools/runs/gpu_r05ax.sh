#!/bin/bash
# round 5: kernel trace of the per-rank step at W = 8 (config 2, rank 0, simulated collectives) -- where the
# 8.8 ms go beyond the kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05ax
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- \
  python3 -u bench.py --no-cpu-baseline --no-files-baseline --no-files-config2 --config3-steps 0 --steps 20 --warmup 2 \
  --sim-world 8 --sim-rank 0 > $O/sim.json 2> $O/sim.err || { tail -n 30 $O/sim.err; exit 1; }
python -c "import json;d=json.load(open('$O/sim.json'));print('cfg2 rank', d['ms_per_step'], d['stages_ms'])"
