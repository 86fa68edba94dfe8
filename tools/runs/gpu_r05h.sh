#!/bin/bash
# round 5: inflate fast tables in registers (readlane) vs LDS: throughput A/B (interleaved), then the inflate tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05h
mkdir -p $O
L=$GRAFT_REPO_ROOT/grid_amd/_lib
for rep in 1 2; do
  for v in vtab lds; do
    if [ $v = lds ]; then export GRID_AMD_LIB=$L/libgridhip_inflate_lds.so; else unset GRID_AMD_LIB; fi
    timeout -k 10 300 python -u tools/bench_inflate.py --bgzf --units --files 256 --json $O/inflate_${v}_$rep.json \
      > $O/inflate_${v}_$rep.log 2>&1 || { tail -n 20 $O/inflate_${v}_$rep.log; exit 1; }
    tail -n 2 $O/inflate_${v}_$rep.log
  done
done
unset GRID_AMD_LIB
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_ingest.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
