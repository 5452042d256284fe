"""Throughput of the simplex (tetrahedral) path on one GPU -- BASELINE configs 4-5.

The reference's simplex configs run on CGAL meshes of cube.off (config 4) and
layers_with_fracture.off (config 5); CGAL is absent, so the meshes are jittered
Kuhn tetrahedralisations:

* cubetask: BASELINE config 4 itself, parseTaskCube (launcher/main.cpp:547-639):
            cube.off at spatial step 0.05, Courant 1, FIXED_FORCE zero everywhere
            and the step traction t < 0.25 ? -1 : 0 on the x <= 0.01 face (--n ignored);
* cube:     the unit cube, n^3 cubes, free surface on every face (the reference's
            parseTaskCgal3d: FIXED_FORCE 0 from an InfiniteArea), pressure sphere;
* fracture: the 0.16 x 0.16 x 0.04 layer of layers_with_fracture.off with its
            tetrahedral fracture carved out, free surface on the box and the fracture;
* layered:  the unit cube split at z = 0.5 into two bodies of different materials
            glued by an ADHESION contact, free surface outside.

A node-step is one mesh vertex advanced one full time step (3 stages, border and
contact correctors included).  Timed: K steps of SimplexEngine.run_steps between
two stream synchronisations, inputs resident on the device.  Prints one JSON line
per workload.

    python scripts/bench_simplex.py [--workloads cubetask,cube,fracture,layered] [--n 64]

Each line carries the step's dependent launches (launches_per_step, counted by
gsx_launch_count) and the launch floor they imply (floor_ms: 1.45-1.9 us per
kernel boundary, MI355X_MICROARCH.md) beside the measured ms_per_step.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(name, n):
    from tests.simplex_spec import FREE_BORDER, cube_task, fracture_task, host_task, layered_task
    if name == "cubetask":
        return cube_task(), ("parseTaskCube (main.cpp:547-639): cube.off at spatial step 0.05 "
                             "(20^3 Kuhn cubes), Courant 1, free surface + the x <= 0.01 traction "
                             "(0, 0, t < 0.25 ? -1 : 0)")
    if name == "cube":
        return host_task(n, 1.0, 0.1, 7, border=FREE_BORDER), f"unit cube, {n}^3 Kuhn cubes"
    if name == "fracture":
        cells = (n, n, max(4, n // 4))
        return fracture_task(cells, 1.0), f"layers_with_fracture.off, {cells} Kuhn cubes"
    if name == "layered":
        return layered_task(n, 1.0), f"two layers + ADHESION contact, {n}^3 Kuhn cubes"
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="cube,fracture,layered")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--lanes", type=int, default=0,
                    help="node-kernel layout (gsx_set_node_lanes): 0 automatic, 1, 8")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step from a gsx_step HIP graph instead of the stage calls")
    ap.add_argument("--fusion", type=int, default=-1,
                    help="gsx_set_stage_fusion: 0 separate launches, 1 border + inner in one, 2 with the "
                         "gradient, -1 (the engine's default) measured per mesh on the first steps")
    a = ap.parse_args()
    from gcm_amd import _gcm_host as H
    for name in a.workloads.split(","):
        t0 = time.perf_counter()
        task, desc = build(name, a.n)
        task.number_of_snaps = 10 ** 6
        e = H.SimplexEngine(task)
        e.set_replay_steps(a.graph)
        e.set_node_lanes(a.lanes)
        e.set_stage_fusion(a.fusion)
        setup = time.perf_counter() - t0
        nv = sum(e.number_of_vertices(b) for b in range(e.number_of_bodies))
        # the automatic fusion choice is made on the first 1 + 2 * 8 steps: warm past it
        warm = max(a.warmup, 20) if a.fusion < 0 else a.warmup
        e.run_steps(warm)
        e.sync()
        l0 = e.launches
        t1 = time.perf_counter()
        e.run_steps(a.steps)
        e.sync()
        dt = time.perf_counter() - t1
        lps = (e.launches - l0) / a.steps
        print(json.dumps({
            "metric": "simplex Mnode-steps/s", "workload": name, "mesh": desc,
            "value": round(nv * a.steps / dt / 1e6, 2), "unit": "Mnode-steps/s",
            "ms_per_step": round(dt / a.steps * 1e3, 4), "vertices": nv,
            "bodies": e.number_of_bodies, "contact_pairs": e.number_of_contact_pairs,
            "steps": a.steps, "warmup": a.warmup, "setup_s": round(setup, 1), "dtype": "f64",
            "graph": a.graph, "lanes": a.lanes, "fusion": a.fusion,
            "fusion_in_effect": e.stage_fusion,
            "fusion_times_ms": [round(v, 4) for v in e.fusion_times_ms] if a.fusion < 0 else None,
            "fused_stages": e.fused_stages,
            # the launch floor: every launch of a step is a dependent kernel boundary on
            # the body's stream; MI355X_MICROARCH.md's price list puts one at 1.45 us
            # (trivial kernels) to 1.7-1.9 us (real streaming kernels)
            "launches_per_step": round(lps, 2),
            "floor_ms": [round(lps * 1.45e-3, 4), round(lps * 1.9e-3, 4)],
            "floor_frac": round(lps * 1.45e-3 / (dt / a.steps * 1e3), 3),
        }), flush=True)


if __name__ == "__main__":
    main()
