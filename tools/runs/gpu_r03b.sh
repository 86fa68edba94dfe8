#!/bin/bash
# round 3: the whole -m gpu suite except the two long full-shape configs (run in r03a)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_configs.py::test_config3_50k_x_3M_streamed \
  --deselect tests/test_gpu_configs.py::test_config4_50k_x_30M_streamed > gpurun_out/r03b_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r03b_pytest.log
exit $rc
