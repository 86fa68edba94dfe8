#!/bin/bash
# round 3: GPU inflate occupancy A/B -- fast literal/length table 2^10 at 5 waves per SIMD (production,
# 18 waves per CU by LDS) vs 2^9 at 6 (24 per CU) vs 2^8 at 7 (28 per CU); 256 BGZF files, one wave per member
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03am
mkdir -p $O
B="--files 256 --bgzf --units"
timeout -k 10 300 python -u tools/bench_inflate.py $B --json $O/inf_l10.json > $O/inf.log 2>&1 &&
GRID_AMD_LIB=$GRAFT_REPO_ROOT/grid_amd/_lib/alt/libgridhip_inf9.so timeout -k 10 300 python -u tools/bench_inflate.py $B --json $O/inf_l9.json >> $O/inf.log 2>&1 &&
GRID_AMD_LIB=$GRAFT_REPO_ROOT/grid_amd/_lib/alt/libgridhip_inf8.so timeout -k 10 300 python -u tools/bench_inflate.py $B --json $O/inf_l8.json >> $O/inf.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_inflate.py $B --json $O/inf_l10b.json >> $O/inf.log 2>&1
rc=$?
grep "text_gbs" $O/inf.log | python -c "import sys,json; [print(json.loads(l)['text_gbs'], json.loads(l)['seconds']) for l in sys.stdin]"
tail -n 3 $O/inf.log
exit $rc
