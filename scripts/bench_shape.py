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
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gcm_amd  # noqa: E402
from gcm_amd.host import isotropic_elastic_matrices  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("shapes", nargs="+")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--rows", type=int, default=0)
ap.add_argument("--bs", type=int, default=2, help="borderSize (ghost depth)")
ap.add_argument("--free", action="store_true", help="free surfaces on all six faces (gcmx_step_faces)")
a = ap.parse_args()
Q = gcm_amd.gcmx.QUANTITY_CODES if hasattr(gcm_amd.gcmx, "QUANTITY_CODES") else None
FREE = None
if a.free:  # ndi.hpp:30-55: the stress components on each face's normal set to zero
    q = Q
    FREE = [[(q["Sxx"], 0.0), (q["Sxy"], 0.0), (q["Sxz"], 0.0)]] * 2 + \
           [[(q["Syy"], 0.0), (q["Sxy"], 0.0), (q["Syz"], 0.0)]] * 2 + \
           [[(q["Szz"], 0.0), (q["Sxz"], 0.0), (q["Syz"], 0.0)]] * 2


def step(c):
    if FREE is not None:
        c.step_faces(0.9, FREE)
    else:
        c.step(0.9)
U, U1, L = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
for sh in a.shapes:
    X, Y, Z = (int(v) for v in sh.split(","))
    c = gcm_amd.Context(3, a.bs, [X, Y, Z], device=0)
    c.set_materials(U[None], U1[None], L[None])
    if a.rows:
        c.set_schedule(gcm_amd.SCHED_AUTO, a.rows)
    c.fill_random([X, Y, Z], 0x5EED)
    for _ in range(2):
        step(c)
    c.sync()
    c.profile(True)
    avgs, walls = [], []
    for _ in range(a.reps):
        c.profile_reset()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step(c)
        c.sync()
        walls.append((time.perf_counter() - t0) / a.steps * 1e3)
        prof = c.profile_read()
        k = prof["fused_xyz"] if "fused_xyz" in prof else max(prof.values(), key=lambda v: v["total_ms"])
        avgs.append(k["total_ms"] / k["launches"])
    ms = sorted(avgs)[len(avgs) // 2]
    n = X * Y * Z
    print(json.dumps({"shape": [X, Y, Z], "bs": a.bs, "free": a.free, "path": c.last_path,
                      "step_ms": round(sorted(walls)[len(walls) // 2], 4), "kernel_ms": round(ms, 4), "frac": round(144 * n / (ms * 1e-3) / 8e12, 4),
                      "ns_per_node": round(ms * 1e6 / n, 4), "kernel": k["kernel"],
                      "alloc": c.layer_info()["alloc"]}), flush=True)
    c.close()
