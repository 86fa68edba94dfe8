#!/bin/bash
# round 5: the cohort split -- its kernels and the chain at world 2/4/8 on one GPU (gloo), the Gram paths after the
# tile-list change, then per-rank timing of both splits (bench --sim-world 8) at config 2 and the config-3 rank shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_cohort.py tests/test_gpu_sharded.py "tests/test_gpu_kernels.py::test_gram_kblocked_multi_slice" \
  "tests/test_gpu_kernels.py::test_gram_variants_multi_slice" > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
B="python -u bench.py --no-cpu-baseline --no-files-baseline --no-files-config2 --config3-steps 0"
for sh in bin cohort; do
  timeout -k 10 200 $B --steps 10 --warmup 2 --sim-world 8 --sim-rank 0 --shard $sh > $O/cfg2_w8_r0_$sh.json 2> $O/cfg2_w8_r0_$sh.err \
    || { tail -n 30 $O/cfg2_w8_r0_$sh.err; exit 1; }
  python -c "import json;d=json.load(open('$O/cfg2_w8_r0_$sh.json'));print('$sh', d['ms_per_step'], d['stages_ms'], d['roofline']['gram_ms'], d.get('sim_collective_bytes_in_per_step'))"
done
timeout -k 10 200 $B --steps 10 --warmup 2 --sim-world 8 --sim-rank 7 --shard cohort > $O/cfg2_w8_r7_cohort.json 2> $O/cfg2_w8_r7_cohort.err \
  || { tail -n 30 $O/cfg2_w8_r7_cohort.err; exit 1; }
python -c "import json;d=json.load(open('$O/cfg2_w8_r7_cohort.json'));print('r7 cohort', d['ms_per_step'], d['roofline']['gram_ms'])"
timeout -k 10 200 $B --steps 10 --warmup 2 --sim-world 8 --sim-rank 0 --shard cohort --piece-mb 512 > $O/cfg2_w8_r0_cohort_p512.json 2> $O/cfg2_w8_r0_cohort_p512.err \
  || { tail -n 30 $O/cfg2_w8_r0_cohort_p512.err; exit 1; }
python -c "import json;d=json.load(open('$O/cfg2_w8_r0_cohort_p512.json'));print('p512', d['ms_per_step'], d['roofline']['gram_ms'])"
for sh in bin cohort; do
  timeout -k 10 400 $B --samples 50000 --steps 2 --warmup 1 --sim-world 8 --sim-rank 0 --shard $sh > $O/cfg3_w8_r0_$sh.json 2> $O/cfg3_w8_r0_$sh.err \
    || { tail -n 30 $O/cfg3_w8_r0_$sh.err; exit 1; }
  python -c "import json;d=json.load(open('$O/cfg3_w8_r0_$sh.json'));print('cfg3 $sh', d['ms_per_step'], d['stages_ms'], d['roofline']['gram_ms'], d.get('sim_collective_bytes_in_per_step'))"
done
