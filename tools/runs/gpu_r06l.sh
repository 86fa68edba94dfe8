#!/bin/bash
# round 6: the driver's bench command after the inflate dispatch fix, the 11-bit selection and
# k_phase4 (from-files headline, K = 20 after 5 warmups), then a kernel-stats profile (csv)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06l
mkdir -p $O
export TMPDIR=/tmp
s0=$(date +%s)
timeout -k 10 590 python3 bench.py --gpus 1 --steps 20 --warmup 5 --keep-files > $O/bench_driver_cmd.json \
  2> $O/bench_driver_cmd.err || { tail -n 40 $O/bench_driver_cmd.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
echo "driver command wall $(( $(date +%s) - s0 )) s"
python3 -c "import json;d=json.load(open('$O/bench_driver_cmd.json'));print('value', d['value'], d['ms_per_step'], d['from_files']['stages_s'], 'chain', d['device_chain']['ms_per_step'], 'frac', d['roofline']['frac'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 3 --warmup 1 \
  --config3-steps 0 --no-cpu-baseline --keep-files > $O/bench_prof.json 2> $O/bench_prof.err \
  || { tail -n 30 $O/bench_prof.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out
find $O/prof -name "*kernel_stats.csv" | head -3
