#!/bin/bash
# round 5: column kernels at 8 waves per SIMD (parity + bench), RCCL collectives of both splits at world 1,
# per-rank timing of both splits (bench --sim-world 8) at config 2 and the config-3 rank shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_depth16.py tests/test_gpu_kernels.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
B="python -u bench.py --no-cpu-baseline --no-files-baseline --no-files-config2 --config3-steps 0"
timeout -k 10 300 $B --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -n 30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['stages_ms'], d['roofline']['gram_ms'])"
for sh in bin cohort; do
  RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 GRID_BENCH_FORCE_DIST=1 timeout -k 10 300 \
    $B --steps 10 --warmup 2 --shard $sh > $O/rccl_w1_$sh.json 2> $O/rccl_w1_$sh.err || { tail -n 30 $O/rccl_w1_$sh.err; exit 1; }
  python -c "import json;d=json.load(open('$O/rccl_w1_$sh.json'));print('rccl w1 $sh', d['ms_per_step'], d['roofline']['gram_ms'], d['config']['parallelism'])"
done
for sh in bin cohort; do
  timeout -k 10 200 $B --steps 10 --warmup 2 --sim-world 8 --sim-rank 0 --shard $sh > $O/sim_cfg2_w8_r0_$sh.json 2> $O/sim_cfg2_$sh.err \
    || { tail -n 30 $O/sim_cfg2_$sh.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sim_cfg2_w8_r0_$sh.json'));print('cfg2 $sh', d['ms_per_step'], d['stages_ms'], d['roofline']['gram_ms'], d.get('sim_collective_bytes_in_per_step'))"
done
timeout -k 10 200 $B --steps 10 --warmup 2 --sim-world 8 --sim-rank 0 --shard cohort --piece-mb 8192 > $O/sim_cfg2_w8_r0_cohort_p8g.json 2> $O/sim_cfg2_p8g.err \
  || { tail -n 30 $O/sim_cfg2_p8g.err; exit 1; }
python -c "import json;d=json.load(open('$O/sim_cfg2_w8_r0_cohort_p8g.json'));print('cfg2 cohort p8g', d['ms_per_step'], d['roofline']['gram_ms'])"
for sh in bin cohort; do
  timeout -k 10 400 $B --samples 50000 --steps 2 --warmup 1 --sim-world 8 --sim-rank 0 --shard $sh --piece-mb 8192 > $O/sim_cfg3_w8_r0_$sh.json 2> $O/sim_cfg3_$sh.err \
    || { tail -n 30 $O/sim_cfg3_$sh.err; exit 1; }
  python -c "import json;d=json.load(open('$O/sim_cfg3_w8_r0_$sh.json'));print('cfg3 $sh', d['ms_per_step'], d['stages_ms'], d['roofline']['gram_ms'], d.get('sim_collective_bytes_in_per_step'))"
done
# zquant7 store-shape microbenchmark (tools/micro/zqstore.hip, built on the CPU side)
timeout -k 10 120 tools/micro/zqstore > $O/zqstore.jsonl 2>&1 || { cat $O/zqstore.jsonl; exit 1; }
cat $O/zqstore.jsonl
