#!/usr/bin/env python3
"""Per-GPU time of one X slab of the 512^3 strong-scaling run, on ONE GPU.

For each slab thickness X (512 / N for N = 1, 2, 4, 8) a [X, 512, 512] context
runs the fused step; with GCMX_SLAB_SCHEDULE=1 in the environment it runs the
multi-GPU step schedule (interior planes on the low-priority stream, 16-row
boundary blocks on the main stream) without a communicator, i.e. everything an
N-rank run does per GPU except the RCCL transfers (which it overlaps).
Also checks the slab step bitwise against the generic per-stage path on a
[64, 512, 512] slab.  One JSON line per size on stdout.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import gcm_amd  # noqa: E402
from gcm_amd import gcmx  # noqa: E402
from gcm_amd.host import isotropic_elastic_matrices  # noqa: E402

U, U1, L = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
N = int(os.environ.get("SLAB_N", "512"))
STEPS = int(os.environ.get("SLAB_STEPS", "20"))


def make(X, path=gcmx.PATH_AUTO, x0=0):
    c = gcm_amd.Context(3, 2, [X, N, N], start=[x0, 0, 0], device=0)
    c.set_materials(U[None], U1[None], L[None])
    c.set_path(path)
    c.fill_random([N, N, N], 0x5EED)
    return c


outs = {}
for name, path in (("fused", gcmx.PATH_FUSED), ("generic", gcmx.PATH_GENERIC)):
    c = make(64, path, x0=128)
    for _ in range(2):
        c.step(0.9)
    outs[name] = c.download()
    c.close()
bad = int(np.sum(outs["fused"] != outs["generic"]))
print(json.dumps({"check": "slab 64x512x512 fused vs generic, 2 steps", "mismatches": bad,
                  "slab_schedule": os.environ.get("GCMX_SLAB_SCHEDULE", "0")}), flush=True)
if bad:
    sys.exit(1)

for ranks in (1, 2, 4, 8):
    X = N // ranks
    c = make(X)
    for _ in range(3):
        c.step(0.9)
    c.sync()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        c.step(0.9)
    c.sync()
    el = time.perf_counter() - t0
    c.profile(True)
    c.profile_reset()
    for _ in range(STEPS):
        c.step(0.9)
    c.sync()
    k = c.profile_read()
    c.profile(False)
    c.close()
    ms = el / STEPS * 1e3
    rate = X * N * N * STEPS / el / 1e6
    print(json.dumps({"ranks": ranks, "slab": [X, N, N], "ms_per_step": round(ms, 4),
                      "Mnode_steps_per_gpu": round(rate, 1),
                      "projected_job_rate_no_comm": round(rate * ranks, 1),
                      "kernels": {n: round(v["total_ms"] / max(1, v["launches"]), 4)
                                  for n, v in k.items()},
                      "slab_schedule": os.environ.get("GCMX_SLAB_SCHEDULE", "0"),
                      "rows": os.environ.get("GCMX_XYZ_ROWS", "auto")}), flush=True)
