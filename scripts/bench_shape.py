#!/usr/bin/env python3
"""One-pass step time of an X x Y x Z grid on one GPU (any shape; bench.py times
N^3): median over repetitions of the library's hipEvent-timed launch average,
fraction of 8 TB/s on 144 B per node-step.  One JSON line per shape.

    python scripts/bench_shape.py 1024,1024,512 [512,512,512 ...] [--steps 5 --reps 3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gcm_amd  # noqa: E402
from gcm_amd.host import isotropic_elastic_matrices  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("shapes", nargs="+")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--rows", type=int, default=0)
a = ap.parse_args()
U, U1, L = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
for sh in a.shapes:
    X, Y, Z = (int(v) for v in sh.split(","))
    c = gcm_amd.Context(3, 2, [X, Y, Z], device=0)
    c.set_materials(U[None], U1[None], L[None])
    if a.rows:
        c.set_schedule(gcm_amd.SCHED_AUTO, a.rows)
    c.fill_random([X, Y, Z], 0x5EED)
    for _ in range(2):
        c.step(0.9)
    c.sync()
    c.profile(True)
    avgs = []
    for _ in range(a.reps):
        c.profile_reset()
        for _ in range(a.steps):
            c.step(0.9)
        c.sync()
        k = c.profile_read()["fused_xyz"]
        avgs.append(k["total_ms"] / k["launches"])
    ms = sorted(avgs)[len(avgs) // 2]
    n = X * Y * Z
    print(json.dumps({"shape": [X, Y, Z], "kernel_ms": round(ms, 4), "frac": round(144 * n / (ms * 1e-3) / 8e12, 4),
                      "ns_per_node": round(ms * 1e6 / n, 4), "kernel": k["kernel"],
                      "alloc": c.layer_info()["alloc"]}), flush=True)
    c.close()
