#!/bin/bash
# round 3: the BASELINE-config tests (configs 1, 3, 4, 5) and the streamed escape list
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="python -u -m pytest -x -v -s --timeout 1200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_configs.py::test_streamed_property_checks_small \
  tests/test_gpu_streamed.py::test_streamed_escapes_reuse_the_list_per_chunk \
  tests/test_gpu_e2e.py::test_config1_100x30k_matches_reference > gpurun_out/r03a_small.log 2>&1 &&
timeout -k 10 400 $T tests/test_gpu_configs.py::test_config3_50k_x_3M_streamed \
  tests/test_gpu_configs.py::test_config5_734_loci_x_50k > gpurun_out/r03a_cfg35.log 2>&1 &&
timeout -k 10 600 $T tests/test_gpu_configs.py::test_config4_50k_x_30M_streamed > gpurun_out/r03a_cfg4.log 2>&1
rc=$?
tail -5 gpurun_out/r03a_*.log
exit $rc
