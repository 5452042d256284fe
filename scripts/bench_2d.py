"""The 2-D step on one GPU: the one-pass k_step2d against the two generic stages.

Workloads (one material (4, 2, 1), Courant 0.9, synthetic parity-random field):

* preset: the reference's 2-D launcher task (parseTask2d, launcher/main.cpp:332-373):
          100 x 50 nodes, borderSize 2 -- launch-bound;
* NxN:    an N x N grid, borderSize 2 (--n, default 8192: 67 M nodes, 2 x 2.7 GB layers).

A node-step is one node advanced one full time step (2 stages).  Timed: K steps
between two stream synchronisations, inputs resident on the device.  For each
path the line carries the kernel's mean duration from HIP events (gcmx_profile)
and its rate on the algorithmic bytes (80 B per node-step for the one-pass
step, 80 B per node-stage for the generic stages) against the 8 TB/s HBM peak.
Prints one JSON line per (workload, path).

    python scripts/bench_2d.py [--n 8192] [--steps 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0


def run(G, gcmx, X, Y, bs, path, steps, warmup, label):
    from gcm_amd.host import isotropic_elastic_matrices
    U, U1, L = isotropic_elastic_matrices(2, 4.0, 2.0, 1.0)
    c = G.Context(2, bs, [X, Y], h=[1.0, 1.0])
    c.set_materials(U[None], U1[None], L[None])
    c.set_path(path)
    c.fill_random([X, Y], 0x5EED)
    tau = 0.9
    for _ in range(warmup):
        c.step(tau)
    c.sync()
    c.profile(True)
    c.profile_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        c.step(tau)
    c.sync()
    el = time.perf_counter() - t0
    prof = c.profile_read()
    c.profile(False)
    kern = {}
    for k, v in prof.items():
        avg = v["total_ms"] / max(1, v["launches"])
        kern[k] = {"kernel": v["kernel"], "avg_ms": round(avg, 5), "launches_per_step": v["launches"] / steps,
                   "GBps": round(v["bytes_per_launch"] / (avg * 1e-3) / 1e9, 1),
                   "frac": round(v["bytes_per_launch"] / (avg * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
    out = {"workload": label, "nodes": X * Y, "bs": bs, "path": c.last_path,
           "ms_per_step": round(el / steps * 1e3, 5),
           "Mnode_steps_per_s": round(X * Y * steps / el / 1e6, 1), "kernels": kern}
    c.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    import gcm_amd as G
    from gcm_amd import gcmx
    for (X, Y, label) in ((100, 50, "preset parseTask2d 100x50"), (a.n, a.n, f"{a.n}x{a.n}")):
        for path in (gcmx.PATH_AUTO, gcmx.PATH_GENERIC):
            print(json.dumps(run(G, gcmx, X, Y, 2, path, a.steps, a.warmup, label)), flush=True)


if __name__ == "__main__":
    main()
