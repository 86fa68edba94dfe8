#!/bin/bash
# round 4: verifier pinned by goldens, config-5 100-sweep oracle check + batch (phase_batch frees
# per group), e2e goldens (step-5 zq hand-off holder), then from-files config 2 and the host read probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_verifier.py tests/test_gpu_e2e.py tests/test_gpu_loci.py \
  "tests/test_gpu_configs.py::test_config5_batch_loci_100_sweeps_vs_oracle" \
  "tests/test_gpu_configs.py::test_config5_734_loci_x_50k" > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 3 $O/pytest.log
GRID_INGEST_TRACE=1 timeout -k 10 600 python -u tools/e2e_files.py --bgzf --reuse --json $O/e2e_files_config2_bgzf.json \
  > $O/e2e.log 2>&1 || { tail -n 30 $O/e2e.log; exit 1; }
grep -E "ingest\]|e2e\]" $O/e2e.log | tail -n 16
timeout -k 10 300 python -u tools/bench_read.py /dev/shm/grid_e2e/mosdepth --gb 8 > $O/read.jsonl 2>&1
rc=$?
cat $O/read.jsonl
rm -rf /dev/shm/grid_e2e
exit $rc
