#!/bin/bash
# round 6: the per-rank W = 8 step's Gram under the launcher's performance knobs (results exact for any
# value): the cost model's choice against every K split over XCDs (GRID_GRAM_KX) and finer K chunks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06u
mkdir -p $O
export TMPDIR=/tmp
for v in default kx1 kx2 kx4 kx8 kc2x default2; do
  case $v in
    kx*) export GRID_GRAM_KX=${v#kx}; unset GRID_GRAM_KC ;;
    kc2x) unset GRID_GRAM_KX; export GRID_GRAM_KC=64 ;;
    *) unset GRID_GRAM_KX GRID_GRAM_KC ;;
  esac
  timeout -k 10 200 python3 bench.py --sim-world 8 --sim-rank 0 --steps 20 --warmup 5 > $O/sim_$v.json 2> $O/sim_$v.err \
    || { tail -n 30 $O/sim_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sim_$v.json'));print('$v', round(d['rank_ms_per_step'],3), 'gram', round(d['roofline']['gram_ms'],3), 'frac', round(d['roofline']['frac'],3))"
done
