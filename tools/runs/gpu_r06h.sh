#!/bin/bash
# round 6: selection histograms shared by keys with one prefix (a pick workgroup per pass),
# two workgroups per CU with 8 values in flight; parity through the select / chain tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_select.py tests/test_gpu_kernels.py tests/test_gpu_sharded.py tests/test_gpu_e2e.py \
  > $O/pytest.log 2>&1 || { tail -n 60 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 200 python3 bench.py --sim-world 8 --sim-rank 0 --steps 20 --warmup 5 \
  > $O/sim_cfg2_w8_r0_bin.json 2> $O/sim.err || { tail -n 30 $O/sim.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/sim_cfg2_w8_r0_bin.json'));print('sim', d['rank_ms_per_step'], d['stages_ms'], d['roofline']['gram_ms'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o sim -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --sim-world 8 --sim-rank 0 --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/$O/sim_prof.json" \
  2> "$GRAFT_REPO_ROOT/$O/sim_prof.err" || { tail -n 20 "$GRAFT_REPO_ROOT/$O/sim_prof.err"; exit 1; }
