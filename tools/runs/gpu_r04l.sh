#!/bin/bash
# round 4: inflate member CRC check (wave per member), 16 KiB parse chunks: inflate/ingest GPU tests,
# the overlay disk's write rate (buffered / O_DIRECT), then the from-files config-2 steps under rocprofv3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_inflate.py tests/test_gpu_ingest.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 3 $O/pytest.log
{ df -h /tmp; for m in buffered fdatasync direct; do
    case $m in direct) f="oflag=direct";; fdatasync) f="conv=fdatasync";; *) f="";; esac
    echo "== $m"; timeout -k 5 120 dd if=/dev/zero of=/tmp/ddtest bs=64M count=96 $f 2>&1 | tail -n 1; rm -f /tmp/ddtest; done; } > $O/disk.txt 2>&1
cat $O/disk.txt
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --generate-only > $O/gen.log 2>&1 || { tail -n 20 $O/gen.log; exit 1; }
GRID_INGEST_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- \
  python3 -u tools/e2e_files.py --bgzf --reuse --json $O/e2e.json > $O/e2e.log 2>&1
rc=$?
rm -rf /dev/shm/grid_e2e
grep -E "e2e\] .*(step4_ingest|step4_write|done in)" $O/e2e.log | tail -n 8
find $O/stats -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/stats -name "*kernel_trace.csv" -exec gzip -c {} \; > $O/kernel_trace.csv.gz
rm -rf $O/stats
exit $rc
