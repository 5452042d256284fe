"""Diagnostic: in-process slab groups with mixed slab widths (some below 4*bs)
under each schedule and fp mode; prints ok / the error per case."""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
os.environ.setdefault("GCMX_LOCAL_WAIT_SECONDS", "10")
import gcm_amd  # noqa: E402
from gcm_amd.host import isotropic_elastic_matrices  # noqa: E402

U, U1, L = isotropic_elastic_matrices(3, 4, 2, 1)
for fp in (gcm_amd.FP_EXACT, gcm_amd.FP_FMA):
    for sched in (gcm_amd.SCHED_BFIRST, gcm_amd.SCHED_XSLAB, gcm_amd.SCHED_SINGLE):
        for xs in ([8, 8, 8], [8, 6, 10], [12, 9, 19], [6, 6]):
            slabs, x0 = [], 0
            for X in xs:
                c = gcm_amd.Context(3, 2, [X, 20, 64], start=[x0, 0, 0])
                c.set_materials(U[None], U1[None], L[None])
                c.fp_mode = fp
                c.fill_random([sum(xs), 20, 64], 7)
                c.set_schedule(sched)
                slabs.append(c)
                x0 += X
            gcm_amd.comm_init_local(slabs)
            t0 = time.time()
            try:
                gcm_amd.local_group_steps(slabs, 0.9, 3)
                r = "ok"
            except Exception as e:
                r = f"ERR {e}"
            print(f"fp {fp} sched {sched} xs {xs}: {r} ({time.time() - t0:.1f}s)", flush=True)
            for c in slabs:
                try:
                    c.close()
                except Exception as e:
                    print("close:", e)
