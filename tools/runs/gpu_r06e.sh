#!/bin/bash
# round 6: (1) the two-literal inflate entries rewritten top-down, A/B against no pairs and against 2^9 / 2^10
# literal tables (6 / 5 waves per SIMD) with pairs; (2) the device chain's per-rank W = 8 step with the phase
# lanes and the column passes on CU-partitioned streams, the one-launch segment pack and the wave-per-row merge
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06e
mkdir -p $O
export TMPDIR=/tmp
L=grid_amd/_lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_sharded.py tests/test_gpu_kernels.py tests/test_gpu_cohort.py tests/test_gpu_ingest.py tests/test_gpu_e2e.py tests/test_gpu_dist_wgs.py \
  > $O/pytest.log 2>&1 || { tail -n 60 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for v in l9 l10; do
  GRID_AMD_LIB=$L/libgridhip_inflate_$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 \
    --timeout-method thread -p no:cacheprovider tests/test_gpu_inflate.py > $O/pytest_inflate_$v.log 2>&1 \
    || { tail -n 40 $O/pytest_inflate_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/pytest_inflate_$v.log)"
done
for k in 1 2; do
  for v in pair nopair l9 l10; do
    lib=$L/libgridhip.so; [ $v != pair ] && lib=$L/libgridhip_inflate_$v.so
    GRID_AMD_LIB=$lib timeout -k 10 200 python -u tools/bench_inflate.py --bgzf --units --files 128 \
      --json $O/inflate_${v}_$k.json > $O/inflate_${v}_$k.log 2>&1 || { tail -n 30 $O/inflate_${v}_$k.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/inflate_${v}_$k.json'));print('$v $k', round(d['text_gbs'],2), 'GB/s')"
  done
done
for cm in "" "--no-cu-mask"; do
  tag=cumask; [ -n "$cm" ] && tag=nocumask
  timeout -k 10 200 python3 bench.py --sim-world 8 --sim-rank 0 --steps 20 --warmup 5 $cm \
    > $O/sim_cfg2_w8_r0_bin_$tag.json 2> $O/sim_$tag.err || { tail -n 30 $O/sim_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sim_cfg2_w8_r0_bin_$tag.json'));print('$tag', d['rank_ms_per_step'], d['stages_ms'])"
done
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --config3-steps 0 --no-cpu-baseline > $O/bench_files.json \
  2> $O/bench_files.err || { tail -n 30 $O/bench_files.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_files.json'));print('files', d['ms_per_step'], d['from_files']['stages_s'], 'chain', d['device_chain']['ms_per_step'])"
