#!/bin/bash
# round 5: where the from-files ingest's wall time goes beyond its kernels -- config 2 from files at threads 16
# under a kernel + memory-copy trace (timestamps of every inflate / parse launch and every H2D), for a GPU-idle
# timeline of step 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05at
mkdir -p $O
export TMPDIR=/tmp
D=/dev/shm/grid_r05at
timeout -k 10 300 python -u tools/e2e_files.py --bgzf --data $D --generate-only --reuse > $O/gen.log 2>&1 \
  || { tail -n 20 $O/gen.log; rm -rf $D; exit 1; }
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- \
  python3 -u tools/e2e_files.py --bgzf --data $D --reuse --threads 16 --json $O/e2e_t16.json \
  > $O/e2e_t16.log 2>&1 || { tail -n 30 $O/e2e_t16.log; rm -rf $D; exit 1; }
rm -rf $D
python -c "import json; d=json.load(open('$O/e2e_t16.json')); print(round(d['steps_4_7_s'],2), {k: round(v,2) for k,v in d['phases_s'].items() if k.startswith('step')})"
find $O/trace -name "*.csv" | head
