#!/usr/bin/env python3
"""Summarise scripts/gpu_counters.sh output: per library variant, the median per
dispatch of every counter of the step kernel (k_fused_xyz / k_step_*), plus
derived figures (effective clock, average L2 read latency, VALU busy)."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

root = sys.argv[1]
for var in sorted(os.listdir(root)):
    d = os.path.join(root, var)
    if not os.path.isdir(d):
        continue
    vals = defaultdict(list)
    dur = []
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "k_fused_xyz" not in k and "k_step_" not in k:
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
            if row["Counter_Name"] == "GRBM_GUI_ACTIVE":
                dur.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    med = {k: statistics.median(v) for k, v in vals.items()}
    print(f"== {var}")
    for k in sorted(med):
        print(f"  {k:40s} {med[k]:.4g}")
    if dur and "GRBM_GUI_ACTIVE" in med:
        t = statistics.median(dur)
        print(f"  dispatch (profiled) {t * 1e3:.3f} ms, effective clock {med['GRBM_GUI_ACTIVE'] / 8 / t / 1e9:.2f} GHz")
    if med.get("TCP_TCC_READ_REQ_sum"):
        print(f"  avg L2 read latency {med['TCP_TCC_READ_REQ_LATENCY_sum'] / med['TCP_TCC_READ_REQ_sum']:.0f} cycles")
    if med.get("SQ_BUSY_CYCLES") and med.get("SQ_ACTIVE_INST_VALU"):
        print(f"  VALU active / wave cycles {med['SQ_ACTIVE_INST_VALU'] / med['SQ_WAVE_CYCLES']:.3f}, "
              f"wait / wave cycles {med['SQ_WAIT_INST_ANY'] / med['SQ_WAVE_CYCLES']:.3f}")
