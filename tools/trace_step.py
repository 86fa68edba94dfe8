"""One step of a rocprofv3 kernel trace as a timeline: start offset, idle gap
before each kernel, duration, queue, name (the step = the kernels from one
k_row_blocks* launch to the next).  python tools/trace_step.py TRACE.csv [which]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else -3
starts = [i for i, x in enumerate(rows) if "k_row_blocks" in x["Kernel_Name"]]
i0, i1 = starts[which], starts[which + 1]
t0 = int(rows[i0]["Start_Timestamp"])
prev, gaps, end = t0, 0, t0
for x in rows[i0:i1]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    gap = s - prev
    if x["Queue_Id"] == rows[i0]["Queue_Id"]:
        gaps += max(gap, 0)
        prev = max(prev, e)
    end = max(end, e)
    print(f"{(s - t0) / 1e3:8.1f} gap {gap / 1e3:7.1f} dur {(e - s) / 1e3:8.1f}  q{x['Queue_Id']} {x['Kernel_Name'][:70]}")
print(f"main queue busy to {(prev - t0) / 1e3:.1f} us, idle gaps {gaps / 1e3:.1f} us; step end {(end - t0) / 1e3:.1f} us")
