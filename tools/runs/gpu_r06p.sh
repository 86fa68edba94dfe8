#!/bin/bash
# round 6: every GPU test on the current build (inflate dispatch, unstructurized uniform branches,
# 11-bit selection, k_phase4), smoke(), then the driver's bench command (from-files headline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests \
  > $O/pytest_gpu_full.log 2>&1 || { tail -n 60 $O/pytest_gpu_full.log; exit 1; }
tail -n 2 $O/pytest_gpu_full.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -n 30 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
s0=$(date +%s)
timeout -k 10 590 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json \
  2> $O/bench_driver_cmd.err || { tail -n 40 $O/bench_driver_cmd.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
echo "driver command wall $(( $(date +%s) - s0 )) s"
python3 -c "import json;d=json.load(open('$O/bench_driver_cmd.json'));print('value', d['value'], d['ms_per_step'], d['from_files']['stages_s'], 'chain', d['device_chain']['ms_per_step'], 'frac', d['roofline']['frac'])"
