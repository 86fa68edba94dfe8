#!/bin/bash
# round 6: k_inflate with two-literal fast-table entries -- the inflate / ingest / e2e tests, then A/B against the
# same kernel without them (libgridhip_inflate_nopair.so): the inflate microbenchmark and the from-files bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_ingest.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 \
  || { tail -n 60 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
NP=grid_amd/_lib/libgridhip_inflate_nopair.so
for k in 1 2; do
  timeout -k 10 300 python -u tools/bench_inflate.py --bgzf --units --files 128 --json $O/inflate_pair_$k.json \
    > $O/inflate_pair_$k.log 2>&1 || { tail -n 30 $O/inflate_pair_$k.log; exit 1; }
  GRID_AMD_LIB=$NP timeout -k 10 300 python -u tools/bench_inflate.py --bgzf --units --files 128 \
    --json $O/inflate_nopair_$k.json > $O/inflate_nopair_$k.log 2>&1 || { tail -n 30 $O/inflate_nopair_$k.log; exit 1; }
  tail -n 1 $O/inflate_pair_$k.log $O/inflate_nopair_$k.log
done
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --config3-steps 0 --no-cpu-baseline --keep-files \
  > $O/bench_pair.json 2> $O/bench_pair.err || { tail -n 30 $O/bench_pair.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
GRID_AMD_LIB=$NP timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --config3-steps 0 --no-cpu-baseline \
  > $O/bench_nopair.json 2> $O/bench_nopair.err || { tail -n 30 $O/bench_nopair.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out
for v in pair nopair; do
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', d['ms_per_step'], d['from_files']['stages_s'])"
done
