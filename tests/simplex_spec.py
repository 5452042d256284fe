"""Shared simplex task builder for the CPU and GPU simplex tests."""
import os

import numpy as np

from oracle import oracle as O
from oracle import simplex as S


def host_task(n=4, courant=1.0, jitter=0.1, seed=7, snaps=3, pressure=1.0, vector=None, border=()):
    """border: Task::borderConditions as (area tuple, "FIXED_FORCE" | "FIXED_VELOCITY",
    [3 functions of t], useForMulticontactNodes)."""
    from gcm_amd import _gcm_host as H
    t = H.Task()
    t.dimensionality = 3
    t.grid = "SIMPLEX"
    t.courant = courant
    t.number_of_snaps = snaps
    t.add_body(0, [1, 1, 1], [0, 0, 0])
    t.set_body_material(0, 4, 2, 1)
    t.calculation_basis = [1, 0, 0, 0, 1, 0, 0, 0, 1]
    t.set_simplex_box([n, n, n], [0, 0, 0], [1, 1, 1], jitter, seed)
    if pressure:
        t.add_initial_quantity(("sphere", 0.3, (0.5, 0.5, 0.5)), "PRESSURE", pressure)
    if vector is not None:
        t.add_initial_vector(("infinite",), list(vector))
    for area, kind, values, multi in border:
        t.add_simplex_border_condition(area, kind, list(values), multi)
    return t


def _contains(area):
    def f(p):
        return bool(O.area_contains(area, np.array([p[0]]), np.array([p[1]]), np.array([p[2]]))[0])
    return f


def oracle_conditions(border):
    return [{"contains": _contains(a), "type": k, "values": list(v), "multi": m}
            for a, k, v, m in border]


def oracle_engine(plans, courant, border=()):
    """The oracle engine on the product's mesh (input data) with its own matrices."""
    U, U1, L = O.isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
    return S.Engine(plans["coords"], plans["cells"], U, U1, L, np.eye(3), courant, plans["pde"],
                    oracle_conditions(border))


ZERO = (lambda t: 0.0,) * 3
FREE_BORDER = [(("infinite",), "FIXED_FORCE", ZERO, True)]   # main.cpp:209-220 (cube task)
# a time-dependent velocity on the x = 0 face, free surface elsewhere (the last
# containing condition wins, Engine.cpp:298-303)
MIXED_BORDER = [(("infinite",), "FIXED_FORCE", ZERO, True),
                (("box", (-1.0, 0.2, 0.2), (0.05, 0.8, 0.8)), "FIXED_VELOCITY",
                 (lambda t: 0.1 * t, lambda t: 0.0, lambda t: -0.05), True)]


# BASELINE config 4: parseTaskCube (launcher/main.cpp:547-639) -- meshes/cube.off
# meshed at spatial step 0.05 (here: the jittered Kuhn box mesh of the unit cube
# at h = 0.05, carved by the .off surface, which keeps every cell), Courant 1,
# FIXED_FORCE zero everywhere and, on the x <= 0.01 face, the traction
# (0, 0, t < 0.25 ? -1 : 0); no initial perturbation (the load drives the wave).
CUBE_OFF = os.path.join(os.path.dirname(__file__), "golden", "cube.off")
CUBE_BORDER = [(("infinite",), "FIXED_FORCE", ZERO, True),
               (("box", (-10.0, -10.0, -10.0), (0.01, 10.0, 10.0)), "FIXED_FORCE",
                (lambda t: 0.0, lambda t: 0.0, lambda t: -1.0 if t < 0.25 else 0.0), True)]


def cube_task(h=0.05, courant=1.0, jitter=0.1, seed=7, snaps=100):
    from gcm_amd import _gcm_host as H
    n = int(round(1.0 / h))
    t = H.Task()
    t.dimensionality = 3
    t.grid = "SIMPLEX"
    t.courant = courant
    t.number_of_snaps = snaps
    t.add_body(0, [1, 1, 1], [0, 0, 0])
    t.set_body_material(0, 4, 2, 1)
    t.calculation_basis = [1, 0, 0, 0, 1, 0, 0, 0, 1]
    t.set_simplex_box([n, n, n], [0, 0, 0], [1, 1, 1], jitter, seed)
    t.set_simplex_domain_off(CUBE_OFF)
    for area, kind, values, multi in CUBE_BORDER:
        t.add_simplex_border_condition(area, kind, list(values), multi)
    return t


# BASELINE config 5: meshes/layers_with_fracture.off -- the 0.16 x 0.16 x 0.04
# layer with a tetrahedral fracture (cavity) inside, free surface everywhere
# (the reference's data file, copied as a fixture into tests/golden/).
FRACTURE_OFF = os.path.join(os.path.dirname(__file__), "golden", "layers_with_fracture.off")


def fracture_task(n=(16, 16, 8), courant=1.0, jitter=0.1, seed=7, border=None, snaps=3):
    from gcm_amd import _gcm_host as H
    t = H.Task()
    t.dimensionality = 3
    t.grid = "SIMPLEX"
    t.courant = courant
    t.number_of_snaps = snaps
    t.add_body(0, [1, 1, 1], [0, 0, 0])
    t.set_body_material(0, 4, 2, 1)
    t.calculation_basis = [1, 0, 0, 0, 1, 0, 0, 0, 1]
    t.set_simplex_box(list(n), [0, 0, 0], [0.16, 0.16, 0.04], jitter, seed)
    t.set_simplex_domain_off(FRACTURE_OFF)
    t.add_initial_quantity(("sphere", 0.03, (0.08, 0.08, 0.02)), "PRESSURE", 1.0)
    for area, kind, values, multi in (FREE_BORDER if border is None else border):
        t.add_simplex_border_condition(area, kind, list(values), multi)
    return t


# Two layers of different isotropic-elastic materials glued by an ADHESION
# contact (ContactCorrectorInRiemannInvariants), free surface outside: per-cell
# body ids by cell centroid (z > 0.5 -> body 1), as the INM mesher assigns them.
LAYER_MATERIALS = {0: (4.0, 2.0, 1.0), 1: (2.0, 1.0, 0.5)}


def layered_task(n=6, courant=1.0, jitter=0.1, seed=7, border=None, snaps=3,
                 materials=LAYER_MATERIALS, inm=None):
    """inm: load the mesh from this INM file (INM_MESHER) instead of the box mesher."""
    from gcm_amd import _gcm_host as H
    t = H.Task()
    t.dimensionality = 3
    t.grid = "SIMPLEX"
    t.courant = courant
    t.number_of_snaps = snaps
    for i, (rho, lam, mu) in sorted(materials.items()):
        t.add_body(i, [1, 1, 1], [0, 0, 0])
        t.set_body_material(i, rho, lam, mu)
    t.calculation_basis = [1, 0, 0, 0, 1, 0, 0, 0, 1]
    if inm is None:
        t.set_simplex_box([n, n, n], [0, 0, 0], [1, 1, 1], jitter, seed)
        t.add_simplex_body_area(("box", (-1, -1, 0.5), (2, 2, 2)), 1)
    else:
        t.set_simplex_inm_mesh(str(inm))
    t.set_contact_condition("ADHESION")
    t.add_initial_quantity(("sphere", 0.3, (0.5, 0.5, 0.3)), "PRESSURE", 1.0)
    t.add_initial_vector(("box", (0.2, 0.2, 0.55), (0.8, 0.8, 0.9)),
                         [0.1, -0.2, 0.3, 0.0, 0.05, 0.0, 0.0, 0.0, 0.0])
    for area, kind, values, multi in (FREE_BORDER if border is None else border):
        t.add_simplex_border_condition(area, kind, list(values), multi)
    return t


def oracle_multi(plans, courant, border=FREE_BORDER, materials=LAYER_MATERIALS):
    bodies = []
    for b in plans["bodies"]:
        U, U1, L = O.isotropic_elastic_matrices(3, *materials[int(b["id"])])
        bodies.append({"id": b["id"], "coords": b["coords"], "cells": b["cells"],
                       "global": b["global"], "U": U, "U1": U1, "L": L, "pde": b["pde"]})
    return S.MultiEngine(bodies, np.eye(3), courant, oracle_conditions(border))


def write_inm(path, points, cells, materials):
    """INM mesh text (InmMeshLoader.hpp:96-172): points, cells with 1-based vertices
    and a material, terminating 0."""
    with open(path, "w") as f:
        f.write(f"{len(points)}\n")
        for p in points:
            f.write(" ".join(repr(float(x)) for x in p) + "\n")
        f.write(f"{len(cells)}\n")
        for c, m in zip(cells, materials):
            f.write(" ".join(str(int(x) + 1) for x in c) + f" {int(m)}\n")
        f.write("0\n")

