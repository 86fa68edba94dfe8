#!/bin/bash
# round 6 final: every GPU test, smoke(), the driver's bench command (from-files headline with the
# from-files CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06z3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests \
  > $O/pytest_gpu_full.log 2>&1 || { tail -n 60 $O/pytest_gpu_full.log; exit 1; }
tail -n 1 $O/pytest_gpu_full.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -n 30 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
s0=$(date +%s)
timeout -k 10 590 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json \
  2> $O/bench_driver_cmd.err || { tail -n 40 $O/bench_driver_cmd.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
echo "driver command wall $(( $(date +%s) - s0 )) s"
python3 -c "import json;d=json.load(open('$O/bench_driver_cmd.json'));print('value', d['value'], d['ms_per_step'], d['from_files']['stages_s'], 'chain', d['device_chain']['ms_per_step'], 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['speedup_vs_cpu_baseline'])"
