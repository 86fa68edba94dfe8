#!/bin/bash
# round 6 final: kernel statistics of a short from-files bench (rocprofv3, csv) and the per-rank W = 8 line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zp
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 3 \
  --warmup 1 --config3-steps 0 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err \
  || { tail -n 30 $O/bench_prof.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out
python3 -c "import json;d=json.load(open('$O/bench_prof.json'));print('prof', d['ms_per_step'], d['from_files']['stages_s'], 'gram_ms', d['roofline']['gram_ms'])"
timeout -k 10 200 python3 bench.py --sim-world 8 --sim-rank 0 --steps 20 --warmup 5 > $O/sim_cfg2_w8_r0_bin.json \
  2> $O/sim.err || { tail -n 30 $O/sim.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/sim_cfg2_w8_r0_bin.json'));print('sim', d['rank_ms_per_step'], d['stages_ms'])"
