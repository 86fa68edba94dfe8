#!/bin/bash
# round 3: inflate fast table 2^8, 7 waves per SIMD (28 waves per CU) -- inflate/ingest/e2e tests,
# 1024 BGZF files GPU-only, from-files config 2 (BGZF); then the Gram's timing knobs with the 16x16x32 ring
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03ao
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_ingest.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 &&
GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/bench_dev_ingest.py --samples 1024 --modes gpu --json $O/dev_ingest_1024.json > $O/dev_ingest.log 2>&1 &&
rm -rf /dev/shm/grid_dev_ingest &&
GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/e2e_files.py --bgzf --json $O/e2e_bgzf.json > $O/e2e_bgzf.log 2>&1
rc=$?
rm -rf /dev/shm/grid_dev_ingest /dev/shm/grid_e2e /tmp/grid_e2e_out
tail -n 3 $O/pytest.log; grep -v "batch files" $O/dev_ingest.log | grep -v generated | tail -n 8
grep "e2e\]" $O/e2e_bgzf.log | grep -v " files$" | tail -n 16; grep "batches done\|gathered" $O/e2e_bgzf.log
[ $rc -eq 0 ] && timeout -k 10 300 python -u tools/bench_gram.py --reps 3 \
  --variants kb21,kb21:LAG=0,kb21:LAG=2,kb21:KX=4,kb21:KX=2,kb21:UF=20,kb21:UF=80 > $O/gram_knobs.log 2>&1
rc2=$?
grep "min" $O/gram_knobs.log
[ $rc -eq 0 ] && exit $rc2
exit $rc
