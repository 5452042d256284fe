#!/usr/bin/env python3
"""Tuning builds with -DGCMX_TX2_DIAG=1 only: run 512^3 fused steps and print the
per-wave phase cycles of k_step_tx2 (s_memtime), summed over blocks and steps."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import gcm_amd  # noqa: E402
from gcm_amd import gcmx  # noqa: E402
from gcm_amd.host import isotropic_elastic_matrices  # noqa: E402

N = int(os.environ.get("N", "512"))
lib = ctypes.CDLL(gcmx.LIB_PATH)
buf = (ctypes.c_ulonglong * 128)()
U, U1, L = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
c = gcm_amd.Context(3, 2, [N, N, N], device=0)
c.set_materials(U[None], U1[None], L[None])
c.fill_random([N, N, N], 0x5EED)
c.step(0.9)
c.sync()
lib.gcmx_diag_tx2(buf)
steps = 5
for _ in range(steps):
    c.step(0.9)
c.sync()
assert lib.gcmx_diag_tx2(buf) == 0
a = np.array(buf[:], dtype=np.float64).reshape(16, 8)
# barrier kernel (GCMX_TX2_NB=0): 1 = barrier 1, 2 = zl writes + barrier 2, 4 = ahead loads;
# NB kernel: 2 = region/edge writes + counter, 6 = ahead loads, 4 = neighbour wait + halo copy
names = ["Y stage", "barrier 1", "zl/rg writes (+barrier 2)", "Z stages+stores", "wait+halo (NB) / ahead loads",
         "X stage", "ahead loads (NB)", "-"]
tot = a.sum(axis=1)
print("per wave-in-block: share of cycles by phase")
for w in range(8):
    print(f"wave {w}: " + "  ".join(f"{names[i]} {a[w, i] / tot[w]:.3f}" for i in range(7)))
pair_rows = (N // 2) * N  # every (x pair, row) once, whatever the chunking
print(f"mean cycles per wave per row: {tot[:8].mean() / (pair_rows * steps):.0f}")
