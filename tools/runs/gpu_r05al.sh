#!/bin/bash
# round 5: k_inflate with 32-bit output positions and fast-loop input window (fewer scalar instructions and SGPR
# spills: 92 -> 59 SGPRs, 11 -> 1 VGPRs spilled): parity (GPU inflate / ingest tests), then throughput against
# the 7-wave build, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${RUN:-r05al}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_ingest.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for r in 1 2; do
  for v in product inflate_w7; do
    L=""; [ $v = inflate_w7 ] && L="GRID_AMD_LIB=grid_amd/_lib/libgridhip_inflate_w7.so"
    env $L timeout -k 10 300 python -u tools/bench_inflate.py --bgzf --units --files 128 --json $O/inflate_${v}_$r.json \
      > $O/inflate_${v}_$r.log 2>&1 || { tail -n 20 $O/inflate_${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/inflate_${v}_$r.json'));print('$v', $r, round(d['text_gbs'],2))"
  done
done
