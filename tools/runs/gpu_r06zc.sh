#!/bin/bash
# round 6: rocprofv3 kernel trace of a from-files bench with the ingest_roofline leg: the leg's last
# k_inflate + k_member_check dispatches against its HIP-event launch times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06zc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 1 \
  --warmup 0 --config3-steps 0 --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err \
  || { tail -n 30 $O/bench_prof.err; rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out; exit 1; }
rm -rf /dev/shm/grid_bench_cfg2 /tmp/grid_bench_cfg2_out
python3 - <<'P'
import csv, glob, json
O = "gpurun_out/r06zc"
tr = glob.glob(f"{O}/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(tr)))
key = lambda r: int(r["Start_Timestamp"])
inf = sorted([r for r in rows if "k_inflate(" in r["Kernel_Name"]], key=key)[-4:]
chk = sorted([r for r in rows if "k_member_check" in r["Kernel_Name"]], key=key)[-4:]
d = json.load(open(f"{O}/bench_prof.json"))
res = {"leg_event_ms": d["ingest_roofline"]["launch_ms_each"],
       "trace_k_inflate_ms": [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in inf],
       "trace_k_member_check_ms": [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in chk],
       "ingest_roofline": d["ingest_roofline"]}
json.dump(res, open(f"{O}/leg_vs_trace.json", "w"), indent=1)
print(json.dumps({k: res[k] for k in ("leg_event_ms", "trace_k_inflate_ms", "trace_k_member_check_ms")}))
P
