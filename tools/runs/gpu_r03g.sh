#!/bin/bash
# round 3 (session 2): restored-tree check -- -m gpu minus the two long configs, smoke,
# bench line + kernel stats, RCCL path at world 1, config-5 loci, device-ingest A/B (BGZF)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_configs.py::test_config3_50k_x_3M_streamed \
  --deselect tests/test_gpu_configs.py::test_config4_50k_x_30M_streamed > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err &&
GRID_BENCH_FORCE_DIST=1 timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_rccl_w1.json 2> $O/bench_rccl_w1.err &&
timeout -k 10 120 python -u bench.py --bins 375000 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_bins375k.json 2> $O/bench_bins375k.err &&
timeout -k 10 200 python -u bench.py --samples 50000 --bins 375000 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_cfg3_rank_w8.json 2> $O/bench_cfg3_rank_w8.err &&
timeout -k 10 200 python -u tools/bench_loci.py --samples 50000 --reps 2 > $O/loci_50k.json 2> $O/loci.err &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/stats -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/stats.log 2>&1) &&
GRID_INGEST_TRACE=1 timeout -k 10 300 python -u tools/bench_dev_ingest.py --samples 256 --json $O/dev_ingest_256.json > $O/dev_ingest.log 2>&1
rc=$?
tail -n 3 $O/pytest.log; tail -n 1 $O/smoke.log; cat $O/bench.json $O/bench_rccl_w1.json $O/bench_bins375k.json $O/loci_50k.json; tail -n 12 $O/dev_ingest.log
exit $rc
