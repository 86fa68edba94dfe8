#!/bin/bash
# round 4: config-5 batched phasing with 1 / 2 / 3 groups in flight (engine.phase_batch streams), loci tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_loci.py > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for f in 1 2 3; do
  timeout -k 10 300 python -u tools/bench_loci.py --loci 734 --samples 50000 --iters 100 --reps 2 --inflight $f \
    > $O/loci_50k_inflight$f.json 2> $O/loci_50k_inflight$f.err || { tail -n 20 $O/loci_50k_inflight$f.err; exit 1; }
  python -c "import json; d=json.load(open('$O/loci_50k_inflight$f.json')); print($f, 'device_ms', round(d['device_ms'],1), 'e2e', round(d['end_to_end_s'],3))"
done
