#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace slice (tuning aid): start / end in us
relative to the slice's first kernel, duration and a short kernel name.

    trace_timeline.py RUN_kernel_trace.csv FIRST COUNT
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
a, n = int(sys.argv[2]), int(sys.argv[3])
rows = rows[a:a + n]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    k = r["Kernel_Name"]
    k = k.split("(")[0].replace("void ", "")[-48:]
    print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {k}")
