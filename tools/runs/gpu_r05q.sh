#!/bin/bash
# round 5: LZ77 device writer at config 2 from files (threads 16, twice; the second reads the step-4 file back:
# every member's CRC checked, the parsed matrix digested), then the writer's kernel trace on a 200-row matrix
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${RUN:-r05q}
mkdir -p $O
export TMPDIR=/tmp
D=/dev/shm/grid_${RUN:-r05q}
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --generate-only --reuse > $O/gen.log 2>&1 \
  || { tail -n 20 $O/gen.log; exit 1; }
for k in 1 2; do
  V=""; [ $k = 2 ] && V="--verify-normalized"
  timeout -k 10 400 python -u tools/e2e_files.py --bgzf --data $D --reuse --threads 16 $V --json $O/e2e_$k.json \
    > $O/e2e_$k.log 2>&1 || { tail -n 30 $O/e2e_$k.log; rm -rf $D; exit 1; }
  python -c "import json; d=json.load(open('$O/e2e_$k.json')); print('run $k', round(d['steps_4_7_s'],2), {k: round(v,2) for k,v in d['phases_s'].items() if k.startswith('step')}, d['outputs'].get('normalized.tsv.gz'), d.get('normalized_readback'))"
done
rm -rf $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -- python3 tools/bench_gzwrite_dev.py --n 200 --reps 1 \
  > $O/gzw_prof.json 2> $O/gzw_prof.err || { tail -n 30 $O/gzw_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/gzw_kernel_stats.csv \;
head -n 14 $O/gzw_kernel_stats.csv | cut -c1-160
