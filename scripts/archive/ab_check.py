#!/usr/bin/env python3
"""A/B helper: 2 steps on the fused path vs the generic (per-stage) path of the
same library, random field, ragged sizes (Z in (256, 512] so tuning builds with
GCMX_TUNE_FAST run it).  Prints 'parity ok' or the mismatch count; exit 1 on a
mismatch."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import gcm_amd  # noqa: E402
from gcm_amd import gcmx  # noqa: E402
from gcm_amd.host import isotropic_elastic_matrices  # noqa: E402

U, U1, L = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
bad = 0
for sz in ([9, 131, 300], [8, 131, 300], [16, 257, 512]):
    outs = {}
    for name, path in (("fused", gcmx.PATH_FUSED), ("generic", gcmx.PATH_GENERIC)):
        c = gcm_amd.Context(3, 2, sz, device=0)
        c.set_materials(U[None], U1[None], L[None])
        c.set_path(path)
        c.fill_random(sz, 0x5EED)
        for _ in range(2):
            c.step(0.9)
        outs[name] = c.download()
        c.close()
    bad += int(np.sum(outs["fused"] != outs["generic"]))
print("parity ok" if bad == 0 else f"PARITY MISMATCH: {bad} values")
sys.exit(0 if bad == 0 else 1)
