#!/bin/bash
# round 5: LZ77 device writer -- parity of the written text (device = host writer, e2e goldens), then its size
# and time on a config-2-like matrix, with a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_gzwrite.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 300 python -u tools/bench_gzwrite_dev.py --n 200 > $O/gzw.json 2> $O/gzw.err || { tail -n 30 $O/gzw.err; exit 1; }
cat $O/gzw.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o gzw -- python -u tools/bench_gzwrite_dev.py --n 200 --reps 1 \
  > $O/gzw_prof.json 2> $O/gzw_prof.err || { tail -n 30 $O/gzw_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/gzw_kernel_stats.csv \;
head -n 12 $O/gzw_kernel_stats.csv
