#!/bin/bash
# round 4: k_inflate at 8 waves per SIMD (64 VGPRs, 2^7 distance fast table; libgridhip_inflate8.so) against
# the product's 7 -- the inflate and device-ingest tests on the variant, then interleaved throughput runs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04w
mkdir -p $O
L8=$GRAFT_REPO_ROOT/grid_amd/_lib/libgridhip_inflate8.so
GRID_AMD_LIB=$L8 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_inflate.py tests/test_gpu_ingest.py > $O/pytest_inflate8.log 2>&1 \
  || { tail -n 40 $O/pytest_inflate8.log; exit 1; }
tail -n 1 $O/pytest_inflate8.log
B="--files 256 --bgzf --units"
for v in 7 8 7 8; do
  lib=$GRAFT_REPO_ROOT/grid_amd/_lib/libgridhip.so
  [ $v = 8 ] && lib=$L8
  GRID_AMD_LIB=$lib timeout -k 10 300 python -u tools/bench_inflate.py $B --json $O/inf_w$v.json >> $O/inf.log 2>&1 \
    || { tail -n 20 $O/inf.log; exit 1; }
  python -c "import json; d=json.load(open('$O/inf_w$v.json')); print('wpe', $v, {k: v for k, v in d.items() if 'gbs' in k or 'GB' in k or k.endswith('_s')})"
done
