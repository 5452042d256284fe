#!/usr/bin/env python3
"""Relative L2 distance of the FMA build of the one-pass step (the product
default, gcmx_set_fp_mode) from the reference path, per configuration, for the
record: small grids against the oracle after 10 steps, the
512^3 bench grid after one step against the exact build (itself bitwise equal
to the oracle, tests/test_gpu_parity.py).  One JSON line per case."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import gcm_amd  # noqa: E402
from gcm_amd.host import isotropic_elastic_matrices  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.helpers import context_for, oracle_body, random_state  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


for bs, sizes, steps in ((2, [6, 24, 512], 10), (2, [16, 32, 64], 10), (1, [8, 12, 64], 10), (3, [9, 7, 100], 10)):
    b = oracle_body(3, bs, sizes)
    random_state(b, seed=sum(sizes), ghosts=False)
    c = context_for(b)
    c.fp_mode = gcm_amd.FP_FMA
    worst = []
    for k in range(steps):
        for s in range(3):
            b.stage(s, 0.9)
        c.step(0.9)
        worst.append(rel(b.inner_view(c.download().reshape(b.pde.shape)), b.inner_view(b.pde)))
    print(json.dumps({"case": f"bs {bs} grid {sizes} random field vs oracle", "steps": steps,
                      "rel_l2_per_step": [float(f"{w:.3e}") for w in worst], "max": max(worst),
                      "kernel_path": c.effective_path}), flush=True)
    c.close()

N = int(os.environ.get("FMA_REPORT_N", "512"))
U, U1, L = isotropic_elastic_matrices(3, 4, 2, 1)
outs = {}
for mode in (gcm_amd.FP_FMA, gcm_amd.FP_EXACT):
    c = gcm_amd.Context(3, 2, [N, N, N])
    c.set_materials(U[None], U1[None], L[None])
    c.fp_mode = mode
    c.fill_random([N, N, N], 0x5EED)
    c.step(0.9)
    outs[mode] = c.download()
    c.close()
d = outs[gcm_amd.FP_FMA] - outs[gcm_amd.FP_EXACT]
print(json.dumps({"case": f"{N}^3 bench grid, one step, FMA vs exact build",
                  "rel_l2": rel(outs[gcm_amd.FP_FMA], outs[gcm_amd.FP_EXACT]),
                  "values_differing": int(np.count_nonzero(d)), "values": int(d.size),
                  "max_abs_diff": float(np.max(np.abs(d)))}), flush=True)
