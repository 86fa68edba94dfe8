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
# column statistics: raw-word software-pipelined row groups (GRID_COL_PF=1, tools build) vs the default
for v in 0 1 0 1; do
  GRID_AMD_LIB=grid_amd/_lib/libgridhip_probes.so GRID_COL_PF=$v timeout -k 10 200 python -u bench.py --steps 10 \
    --warmup 2 --no-cpu-baseline --config3-steps 0 --no-files-config2 > $O/colpf$v.json 2> $O/colpf$v.err \
    || { tail -n 20 $O/colpf$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/colpf$v.json')); print('PF', $v, d['ms_per_step'], d['stages_ms']['col_stats'])"
done
