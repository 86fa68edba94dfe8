#!/bin/bash
# round 5: full GPU pass of the tree (cohort split, ingest changes, buffer release, writer slot tag), smoke, the RCCL
# collectives of both splits at world 1 (GRID_BENCH_FORCE_DIST), per-rank timing of both splits re-run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { tail -n 40 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
grep -c "Exception ignored" $O/pytest_gpu.log || true
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -n 20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
B="python -u bench.py --no-cpu-baseline --no-files-baseline --no-files-config2 --config3-steps 0"
for sh in bin cohort; do
  GRID_BENCH_FORCE_DIST=1 timeout -k 10 300 $B --steps 10 --warmup 2 --shard $sh > $O/rccl_w1_$sh.json 2> $O/rccl_w1_$sh.err \
    || { tail -n 30 $O/rccl_w1_$sh.err; exit 1; }
  python -c "import json;d=json.load(open('$O/rccl_w1_$sh.json'));print('rccl w1 $sh', d['ms_per_step'], d['roofline']['gram_ms'], d['config']['parallelism'])"
done
for sh in bin cohort; do
  timeout -k 10 200 $B --steps 10 --warmup 2 --sim-world 8 --sim-rank 0 --shard $sh > $O/sim_cfg2_w8_r0_$sh.json 2> $O/sim_cfg2_$sh.err \
    || { tail -n 30 $O/sim_cfg2_$sh.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sim_cfg2_w8_r0_$sh.json'));print('cfg2 $sh', d['ms_per_step'], d['roofline']['gram_ms'], d.get('sim_collective_bytes_in_per_step'))"
done
timeout -k 10 200 $B --steps 10 --warmup 2 --sim-world 8 --sim-rank 0 --shard cohort --piece-mb 8192 > $O/sim_cfg2_w8_r0_cohort_p8g.json 2> $O/sim_cfg2_p8g.err \
  || { tail -n 30 $O/sim_cfg2_p8g.err; exit 1; }
python -c "import json;d=json.load(open('$O/sim_cfg2_w8_r0_cohort_p8g.json'));print('cfg2 cohort p8g', d['ms_per_step'], d['roofline']['gram_ms'])"
for sh in bin cohort; do
  timeout -k 10 400 $B --samples 50000 --steps 2 --warmup 1 --sim-world 8 --sim-rank 0 --shard $sh --piece-mb 8192 > $O/sim_cfg3_w8_r0_$sh.json 2> $O/sim_cfg3_$sh.err \
    || { tail -n 30 $O/sim_cfg3_$sh.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sim_cfg3_w8_r0_$sh.json'));print('cfg3 $sh', d['ms_per_step'], d['stages_ms'], d['roofline']['gram_ms'], d.get('sim_collective_bytes_in_per_step'))"
done
