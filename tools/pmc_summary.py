"""Summarise rocprofv3 --pmc CSV output per kernel (sum of counters over
dispatches, mean duration from the kernel trace).

    python tools/pmc_summary.py gpurun_out/pmc1 [gpurun_out/pmc2 ...] [--filter gram]
"""
import argparse
import collections
import csv
import glob
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--filter", default="gram")
a = ap.parse_args()


def short(name):
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:60]


for d in a.dirs:
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if a.filter in r["Kernel_Name"]:
                k = short(r["Kernel_Name"])
                cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*_kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if a.filter in r["Kernel_Name"]:
                dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k in sorted(set(cnt) | set(dur)):
        n = max(len(disp[k]), 1)
        ms = sum(dur[k]) / max(len(dur[k]), 1)
        vals = ", ".join(f"{c}={v / n:.4g}" for c, v in sorted(cnt[k].items()))
        print(f"{os.path.basename(d)} {k}: {ms:.3f} ms/dispatch ({len(dur[k])}) {vals}")
