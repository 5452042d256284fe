"""Diagnostic (lease Q): which nodes of the z-split face step differ from the
oracle, for subsets of the failing case's conditions."""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "../.."))
os.environ["GCMX_FP"] = "exact"
from tests.helpers import context_for, random_state  # noqa: E402
from tests.test_gpu_faces import face_body, faces_at, free  # noqa: E402

ALL = {"ypl": (1, 1, free(1, lambda t: 0.3 * math.sin(2 * t))),
       "zmi": (2, -1, free(2, lambda t: -0.2 + 0.1 * t)),
       "ymi": (1, -1, {"Vy": lambda t: 0.1, "Sxy": lambda t: 0.0}),
       "xmi": (0, -1, {"Vx": lambda t: 0.05})}
for combo in (["ypl", "zmi", "ymi", "xmi"], ["xmi"], ["zmi"], ["ymi"], ["ypl"], ["ypl", "zmi", "ymi"]):
    for Z in (1024, 512):
        conds = [ALL[k] for k in combo]
        sizes = [6, 10, Z]
        b = face_body(3, 2, sizes, conds)
        random_state(b, seed=len("z1024_some") + 1024, ghosts=False)
        ctx = context_for(b)
        for s in range(3):
            b.apply_border(s, 0.0)
            b.stage(s, 0.9)
        ctx.step_faces(0.9, faces_at(3, conds, 0.0))
        got = b.inner_view(ctx.download().reshape(b.pde.shape))
        want = b.inner_view(b.pde)
        d = np.argwhere(got != want)
        msg = "ok" if len(d) == 0 else (f"{len(d)} differ; x {sorted(set(d[:, 0].tolist()))} y {sorted(set(d[:, 1].tolist()))} "
                                        f"z {d[:, 2].min()}..{d[:, 2].max()} ({len(set(d[:, 2].tolist()))} cols) comps {sorted(set(d[:, 3].tolist()))}")
        print(combo, Z, ctx.last_path, msg, flush=True)
        ctx.close()
