#!/bin/bash
# round 3: the two full-shape configs back to back in one process (the OOM of r03n: the config-3
# chain's buffers outlived its test), then from-files config 2 with BGZF all on the GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_configs.py::test_config3_50k_x_3M_streamed tests/test_gpu_configs.py::test_config4_50k_x_30M_streamed \
  > $O/pytest_cfg34.log 2>&1 &&
GRID_INGEST_TRACE=1 timeout -k 10 400 python -u tools/e2e_files.py --bgzf --json $O/e2e_bgzf.json > $O/e2e_bgzf.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e /tmp/grid_e2e_out
tail -n 3 $O/pytest_cfg34.log; grep "e2e\]" $O/e2e_bgzf.log | grep -v " files$" | tail -n 16; grep "batches done\|gathered" $O/e2e_bgzf.log
exit $rc
