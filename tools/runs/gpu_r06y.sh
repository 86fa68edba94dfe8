#!/bin/bash
# round 6: member CRC check with per-lane contiguous 1 KiB chunks -- parity (inflate / ingest tests,
# corrupt members) and A/B of the inflate + check rate against the committed kernels (inflate_ref)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06y
mkdir -p $O
export TMPDIR=/tmp
L=grid_amd/_lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_ingest.py tests/test_gpu_select.py > $O/pytest.log 2>&1 || { tail -n 60 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
for k in 1 2; do
  for v in crc ref; do
    lib=$L/libgridhip.so; [ $v != crc ] && lib=$L/libgridhip_inflate_$v.so
    GRID_AMD_LIB=$lib timeout -k 10 200 python -u tools/bench_inflate.py --bgzf --units --files 128 \
      --json $O/inflate_${v}_$k.json > $O/inflate_${v}_$k.log 2>&1 || { tail -n 30 $O/inflate_${v}_$k.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/inflate_${v}_$k.json'));print('$v $k', round(d['text_gbs'],2), 'GB/s')"
  done
done
