#!/bin/bash
# round 4: GPU sharded worlds 2/3/4/8 (ranks sharing the GPU, gloo), then the
# from-files config-2 run on the current tree (libdeflate cohort generator)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_sharded.py > $O/pytest_sharded.log 2>&1 || { tail -n 30 $O/pytest_sharded.log; exit 1; }
tail -n 3 $O/pytest_sharded.log
df -h /dev/shm /tmp > $O/df.txt 2>&1
nproc >> $O/df.txt
GRID_INGEST_TRACE=1 timeout -k 10 600 python -u tools/e2e_files.py --bgzf --json $O/e2e_files_config2_bgzf.json \
  > $O/e2e.log 2>&1
rc=$?
tail -n 5 $O/e2e.log
exit $rc
