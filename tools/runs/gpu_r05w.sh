#!/bin/bash
# round 5: what bounds k_inflate -- scalar-unit issue or latency? SQ instruction / activity counters of the BGZF
# member inflate (bench_inflate --bgzf --units), one PMC pass, beside the plain timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${RUN:-r05w}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_inflate.py --bgzf --units --files 128 --json $O/inflate.json > $O/inflate.log 2>&1 \
  || { tail -n 20 $O/inflate.log; exit 1; }
tail -n 3 $O/inflate.log
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv \
  --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $O/pmc -- python3 tools/bench_inflate.py --bgzf --units --files 128 > $O/pmc.log 2>&1 || { tail -n 20 $O/pmc.log; exit 1; }
find $O/pmc -name "*counter_collection.csv" -exec cp {} $O/pmc_counters.csv \;
python3 - <<PY
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open("$O/pmc_counters.csv")):
    if "inflate" in r["Kernel_Name"]:
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    print(k, dict(v))
PY
