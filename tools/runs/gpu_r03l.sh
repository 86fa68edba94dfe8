#!/bin/bash
# round 3: where the device ingest's time goes at 1024 BGZF files (timestamps); config-5 batch pipeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_loci.py tests/test_gpu_configs.py::test_config5_734_loci_x_50k > $O/pytest.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_loci.py --samples 50000 --reps 2 > $O/loci_50k.json 2> $O/loci.err &&
GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/bench_dev_ingest.py --samples 1024 --modes model,host --json $O/dev_ingest_1024.json > $O/dev_ingest.log 2>&1
rc=$?
rm -rf /dev/shm/grid_dev_ingest
tail -n 3 $O/pytest.log; cat $O/loci_50k.json; grep -v "batch files" $O/dev_ingest.log | tail -n 40
exit $rc
