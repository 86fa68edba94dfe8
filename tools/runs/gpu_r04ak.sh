#!/bin/bash
# round 4: the wave-parallel CRC fold -- writer / ingest / e2e tests, then the from-files config-2 steps under rocprofv3 (kernel statistics of the ingest with a
# quarter of the files on the host threads, the device writer, steps 5-7)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ak
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gzwrite.py tests/test_gpu_ingest.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 \
  || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --generate-only > $O/gen.log 2>&1 || { tail -n 20 $O/gen.log; exit 1; }
GRID_INGEST_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- \
  python3 -u tools/e2e_files.py --bgzf --reuse --json $O/e2e.json > $O/e2e.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
grep -E "e2e\] .*(step4_ingest|step4_write|done in)" $O/e2e.log | tail -n 8
exit $rc
