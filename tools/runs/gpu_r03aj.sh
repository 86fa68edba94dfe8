#!/bin/bash
# round 3: per-rank work of the W = 8 projections with the 16x16x32 Gram: config 2 at 1/8 of the
# bins (3,202 x 375,000) and config 3 at 1/8 (50,000 x 375,000, resident)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03aj
mkdir -p $O
timeout -k 10 200 python -u bench.py --bins 375000 --steps 20 --warmup 3 --no-cpu-baseline --config3-steps 0 > $O/bins375k.json 2> $O/bins375k.err &&
timeout -k 10 300 python -u bench.py --samples 50000 --bins 375000 --steps 3 --warmup 1 --no-cpu-baseline --config3-steps 0 > $O/cfg3_rank_w8.json 2> $O/cfg3_rank_w8.err
rc=$?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03aj/*.json")):
    d = json.load(open(f)); s = d.get("stages_ms", {})
    print(f.split("/")[-1], round(d["ms_per_step"], 3), s, d["roofline"]["gram_ms"], round(d["roofline"]["executed_frac"], 3))
PY
exit $rc
