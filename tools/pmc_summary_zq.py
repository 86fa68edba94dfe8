"""Per-wave SQ instruction counts per kernel from a rocprofv3 --pmc directory."""
import collections
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*_counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
nd = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"][:48]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    nd[k].add(r["Dispatch_Id"])
for k, v in agg.items():
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    w = v["SQ_WAVES"]
    print(f"{k} x{len(nd[k])}: waves {w / len(nd[k]):.0f}, per wave VALU {v['SQ_INSTS_VALU'] / w:.0f} "
          f"SALU {v['SQ_INSTS_SALU'] / w:.0f} VMEM rd {v['SQ_INSTS_VMEM_RD'] / w:.1f} wr {v['SQ_INSTS_VMEM_WR'] / w:.1f}, "
          f"cycles/wave {v['SQ_WAVE_CYCLES'] / w:.0f}")
