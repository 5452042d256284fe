"""Throughput of a physical cubic run: free surfaces on all six faces (cubic
BorderConditions, engine/cubic/BorderConditions.hpp:81-114), optionally the
Maxwell viscosity ODE (rheology/ode/MaxwellViscosityOde.hpp), through the C++
engine (cubic::Engine<3>::nextTimeStep: border fill -> stage -> swap per axis,
then the ODEs).  The conditions cover whole faces, so the engine runs each step
as one gcmx_step_faces call: the one-pass kernel with the y/z ghost rows and
columns formed in registers / LDS and the x faces filled in memory first.

    python scripts/bench_physics.py [--n 256] [--steps 10] [--maxwell]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FACE_FORCE = {0: ["Sxx", "Sxy", "Sxz"], 1: ["Sxy", "Syy", "Syz"], 2: ["Sxz", "Syz", "Szz"]}


def task(n, maxwell, layers=False, free=True, xbodies=1, axis=0, partial=False):
    from gcm_amd import _gcm_host as H
    t = H.Task()
    t.dimensionality = 3
    t.border_size = 2
    t.h = [1.0, 1.0, 1.0]
    t.courant = 0.9
    t.number_of_snaps = 10 ** 6
    if xbodies > 1:  # the domain as bodies stacked along `axis`: contacts (engine: one pass;
        w = n // xbodies  # along y / z the engine runs them as one stack)
        for k in range(xbodies):
            sz, st = [n, n, n], [0, 0, 0]
            sz[axis], st[axis] = w, k * w
            t.add_body(k, sz, st)
    else:
        t.add_body(0, [n, n, n], [0, 0, 0])
    t.set_default_material(4.0, 2.0, 1.0, tau0=50.0 if maxwell else 0.0)
    if layers:  # a second material in the upper half along x (TestEngine.cpp:139-296's two layers)
        t.add_material(("box", (n / 2 - 0.5, -1, -1), (2 * n, 2 * n, 2 * n)), 2.0, 1.0, 0.5,
                       tau0=40.0 if maxwell else 0.0, number=1)
    t.add_initial_quantity(("sphere", n / 4, (n / 2, n / 2, n / 2)), "PRESSURE", 10.0)
    for d, qs in FACE_FORCE.items():  # free surface: zero traction on both faces of axis d
        if free:
            t.add_border_condition(0, d, ("infinite",), {q: (lambda time: 0.0) for q in qs})
    if free and partial:  # a condition over part of face y- (x < n/2): per-node face maps
        t.add_border_condition(0, 1, ("box", (-1, -1, -1), (n / 2 - 0.5, 0.5, n + 1)),
                               {"Vy": (lambda time: -0.1)})
    if maxwell:
        t.add_ode(0, "MAXWELL_VISCOSITY")
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--maxwell", action="store_true")
    ap.add_argument("--layers", action="store_true",
                    help="two materials (per-node material ids: the heterogeneous path)")
    ap.add_argument("--xbodies", type=int, default=1,
                    help="split the domain into this many bodies along x (contacts along x)")
    ap.add_argument("--axis", type=int, default=0, choices=[0, 1, 2],
                    help="the axis --xbodies stacks the bodies along")
    ap.add_argument("--partial", action="store_true",
                    help="free surfaces plus a condition over half of face y- (partial face)")
    ap.add_argument("--free", action=argparse.BooleanOptionalAction, default=True,
                    help="free surfaces on all faces (--no-free: ghosts stay zero)")
    a = ap.parse_args()
    from gcm_amd import _gcm_host as H
    e = H.Engine(task(a.n, a.maxwell, a.layers, a.free and a.xbodies == 1, a.xbodies, a.axis, a.partial))
    free = a.free and a.xbodies == 1
    nb = max(1, a.xbodies)

    def sync_all():
        for b in range(nb):
            e.sync(b)
    e.run_steps(a.warmup)
    sync_all()
    t0 = time.perf_counter()
    e.run_steps(a.steps)
    sync_all()
    dt = time.perf_counter() - t0
    print(json.dumps({
        "metric": "Mnode-steps/s, cubic engine" + (" with free surfaces" if free else "") +
                  (" + Maxwell ODE" if a.maxwell else "") + (", two materials" if a.layers else "") +
                  (" + a condition over half of face y-" if free and a.partial else "") +
                  (f", {nb} bodies along {'xyz'[a.axis]} with contacts" if nb > 1 else ""),
        "value": round(a.n ** 3 * a.steps / dt / 1e6, 1), "unit": "Mnode-steps/s",
        "ms_per_step": round(dt / a.steps * 1e3, 4), "n": a.n, "steps": a.steps,
        "path": e.path(0), "last_path": [e.last_path(b) for b in range(nb)], "ode_fused": e.ode_fused(0),
        "dtype": "f64"}), flush=True)


if __name__ == "__main__":
    main()
