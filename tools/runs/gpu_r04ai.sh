#!/bin/bash
# round 4: the Gram's K split at config 2 (3,202 x 2,699,999 selected: 42,188 K-steps) --
# the cost model's choice against forced K-range counts (GRID_GRAM_KX) and chunk counts (GRID_GRAM_KC)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ai
mkdir -p $O
for c in "- -" "8 -" "4 -" "2 -" "1 -" "- -" "4 -"; do
  set -- $c
  env_=""
  [ "$1" != "-" ] && env_="$env_ GRID_GRAM_KX=$1"
  [ "$2" != "-" ] && env_="$env_ GRID_GRAM_KC=$2"
  tag=kx$1_kc$2
  env $env_ timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline \
    --config3-steps 0 --no-files-config2 > $O/g_$tag.json 2> $O/g_$tag.err || { tail -n 20 $O/g_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/g_$tag.json')); print('$tag', round(d['ms_per_step'],3), round(d['roofline']['gram_ms'],3))"
done
