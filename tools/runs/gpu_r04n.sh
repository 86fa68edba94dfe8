#!/bin/bash
# round 4: device writer with O_DIRECT batches -- writer + e2e GPU tests, the from-files config-2 run,
# then config-5 batched phasing with 1 / 3 groups in flight
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gzwrite.py tests/test_gpu_e2e.py tests/test_gpu_loci.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 3 $O/pytest.log
GRID_INGEST_TRACE=1 timeout -k 10 600 python -u tools/e2e_files.py --bgzf --json $O/e2e_files_config2_bgzf.json \
  > $O/e2e.log 2>&1 || { tail -n 30 $O/e2e.log; exit 1; }
grep -E "e2e\] .*(step4_ingest|step4_write|done in)" $O/e2e.log | tail -n 8
for f in 1 3; do
  timeout -k 10 300 python -u tools/bench_loci.py --loci 734 --samples 50000 --iters 100 --reps 2 --inflight $f \
    > $O/loci_50k_inflight$f.json 2> $O/loci_50k_inflight$f.err || { tail -n 20 $O/loci_50k_inflight$f.err; exit 1; }
  python -c "import json; d=json.load(open('$O/loci_50k_inflight$f.json')); print($f, 'device_ms', round(d['device_ms'],1), 'e2e', round(d['end_to_end_s'],3))"
done
# bench.py --gpus 8 rehearsal, 8 ranks sharing the one GPU over gloo, reduced shape
GRID_BENCH_SHARE_GPU=1 GRID_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 8 --steps 3 --warmup 1 \
  --samples 1024 --bins 524288 --hbm-budget-gb 20 --no-cpu-baseline --config3-steps 0 \
  > $O/bench_gpus8_share.json 2> $O/bench_gpus8_share.err || { tail -n 30 $O/bench_gpus8_share.err; exit 1; }
python -c "import json; L=open('$O/bench_gpus8_share.json').read().splitlines(); assert len(L)==1, L; d=json.loads(L[0]); print('gpus8 rehearsal', d['n_gpus'], d['value'], d['ms_per_step'])"
