#!/usr/bin/env python3
"""Kernel durations and idle gaps of a rocprofv3 kernel trace (tuning aid).

    trace_gaps.py RUN_kernel_trace.csv [SKIP]

Per kernel name: launches, mean duration; then the idle time between the end of
one kernel and the start of the next (GPU idle when no kernel overlaps), summed
over the trace after the first SKIP kernels, and the wall span.  A per-step wall
time well above the kernels' sum shows up here as gap time.
"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[int(sys.argv[2]) if len(sys.argv) > 2 else 0:]
dur = defaultdict(list)
gaps = []
busy_until = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = r["Kernel_Name"]
    n = n.split("(")[0][-60:]
    dur[n].append((e - s) / 1e3)
    if busy_until is not None and s > busy_until:
        gaps.append((s - busy_until) / 1e3)
    busy_until = e if busy_until is None else max(busy_until, e)
for n, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{len(d):6d}  {sum(d) / len(d):10.1f} us  {n}")
span = (busy_until - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"span {span:.1f} us, kernels {sum(sum(d) for d in dur.values()):.1f} us, "
      f"idle gaps {sum(gaps):.1f} us over {len(gaps)} gaps (max {max(gaps) if gaps else 0:.1f} us)")
