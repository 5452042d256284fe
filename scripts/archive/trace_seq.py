#!/usr/bin/env python3
"""Print the kernel sequence (name:duration us) of a rocprofv3 kernel trace: argv[1]
= run_kernel_trace.csv, argv[2:4] = slice bounds."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = []
for r in rows:
    n = r["Kernel_Name"]
    n = n.split("(")[1].split("::")[-1] if "::" in n else n[:20]
    seq.append(f"{n}:{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000:.1f}")
a, b = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (0, len(seq))
print(" ".join(seq[a:b]))
