"""Whole-face cubic border conditions on the device (gcmx_step_faces) and the
device-resident face-node lists (gcmx_border_nodes_create / gcmx_border_apply),
bitwise against the oracle's BorderConditions::apply + stage sequence
(engine/cubic/BorderConditions.hpp:81-114, Engine.cpp:90-121).

The one-pass step forms the ghost rows / columns of the intermediate Y and Z
stages from mirrored X / Y results (kernels_xyz.hip, k_step_tx2<FACES>); these
tests check it against the reference semantics, in which every stage's ghosts
are written into the intermediate layer in memory before the stage runs."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import assert_same, assert_same_inner, context_for, random_state
from tests.taskspec import host_task, oracle_task, spec

pytestmark = pytest.mark.gpu

QCODE = {"Vx": 2, "Vy": 3, "Vz": 4, "Sxx": 5, "Sxy": 6, "Sxz": 7, "Syy": 8, "Syz": 9, "Szz": 10,
         "PRESSURE": 12}
FREE = {0: ("Sxx", "Sxy", "Sxz"), 1: ("Syy", "Sxy", "Syz"), 2: ("Szz", "Sxz", "Syz")}  # ndi.hpp:30-55


@pytest.fixture(scope="module")
def G():
    import gcm_amd
    gcm_amd.lib()
    return gcm_amd


def face_area(D, sizes, axis, side):
    """An axis-aligned box holding exactly the nodes of one face (h = 1, start 0;
    the other axes unbounded for any grid here, rows of 1024 included)."""
    lo = [-1e6] * 3
    hi = [1e6] * 3
    c = 0.0 if side < 0 else float(sizes[axis] - 1)
    lo[axis], hi[axis] = c - 0.5, c + 0.5
    return ("box", tuple(lo), tuple(hi))


def face_body(D, bs, sizes, conditions):
    """conditions: list of (axis, side or 0 for both faces, {quantity: f(t)})."""
    bcs = []
    for axis, side, vals in conditions:
        area = ("infinite",) if side == 0 else face_area(D, sizes, axis, side)
        bcs.append(O.BorderCondition(axis, area, vals))
    t = O.Task(D=D, border_size=bs, h=[1.0] * D, cubics={0: (list(sizes), [0] * D)}, courant=0.9,
               default_material=O.Material(4.0, 2.0, 1.0), number_of_snaps=1,
               border_conditions={0: bcs})
    return O.Engine(t).bodies[0]


def faces_at(D, conditions, time):
    """gcmx_step_faces argument: per face the last condition covering it, its
    quantities in the reference's std::map order evaluated at `time`."""
    faces = [None] * (2 * D)
    for axis, side, vals in conditions:
        lst = sorted(vals.items(), key=lambda kv: O.QUANTITY_ORDER.index(kv[0]))
        entry = [(QCODE[q], f(time)) for q, f in lst]
        for s in ((0, 1) if side == 0 else ((0,) if side < 0 else (1,))):
            faces[2 * axis + s] = entry
    return faces


def free(axis, normal=lambda t: 0.0):
    q = FREE[axis]
    return {q[0]: normal, q[1]: lambda t: 0.0, q[2]: lambda t: 0.0}


FACE_CASES = {
    # free surfaces on all six faces, odd X, Z = 70 (idle lanes), Courant 0.9
    "free_all": (2, [9, 40, 70], [(0, 0, free(0)), (1, 0, free(1)), (2, 0, free(2))], 0.9, "fused"),
    # some faces only, time-dependent normal force on y+ and z-, Z = ZT (no idle lanes)
    "some_faces": (2, [8, 30, 64], [(1, 1, free(1, lambda t: 0.3 * math.sin(2 * t))),
                                    (2, -1, free(2, lambda t: -0.2 + 0.1 * t)),
                                    (0, -1, {"Vx": lambda t: 0.05})], 0.9, "fused"),
    # an overriding later condition on one face (the last one covering a face wins)
    "override": (2, [10, 22, 33], [(1, 0, free(1)), (1, -1, {"Vy": lambda t: 0.1, "Sxy": lambda t: 0.0}),
                                   (2, 0, {"Vz": lambda t: -0.3})], 0.9, "fused"),
    # borderSize 1
    "bs1": (1, [7, 12, 20], [(0, 0, free(0)), (1, 0, free(1)), (2, 0, free(2))], 0.9, "fused"),
    # Courant 1.5 with borderSize 2: floor(q) = 1 on the fast waves (no shared x differences)
    "courant15": (2, [10, 12, 16], [(1, 0, free(1)), (2, 1, free(2, lambda t: 0.5))], 1.5, "fused"),
    # PRESSURE on a y face: its trace needs node-only components -> per-stage path
    "pressure_y": (2, [6, 20, 40], [(1, -1, {"PRESSURE": lambda t: 0.25}), (2, 0, free(2))], 0.9, "split"),
    # PRESSURE on an x face is filled in memory: still one pass
    "pressure_x": (2, [6, 20, 40], [(0, 1, {"PRESSURE": lambda t: 0.25}), (2, 0, free(2))], 0.9, "fused"),
    # rows of 1024: the z split (two 512-lane parts, the cut columns by k_zseam)
    # with the y faces in both kernels and the z faces in the first / last part
    "z1024_free_all": (2, [5, 12, 1024], [(0, 0, free(0)), (1, 0, free(1)), (2, 0, free(2))], 0.9, "fused"),
    "z1024_some": (2, [6, 10, 1024], [(1, 1, free(1, lambda t: 0.3 * math.sin(2 * t))),
                                      (2, -1, free(2, lambda t: -0.2 + 0.1 * t)),
                                      (1, -1, {"Vy": lambda t: 0.1, "Sxy": lambda t: 0.0}),
                                      (0, -1, {"Vx": lambda t: 0.05})], 0.9, "fused"),
    "z1024_bs1": (1, [4, 8, 1024], [(0, 0, free(0)), (1, 0, free(1)), (2, 0, free(2))], 0.9, "fused"),
    # floor(q) = 1: no z split, so the per-stage path
    "z1024_courant15": (2, [4, 8, 1024], [(1, 0, free(1)), (2, 0, free(2))], 1.5, "split"),
    # 512 blocks on 256 CUs: the two-generation row split (old blocks 20 rows,
    # young 12) with y faces on the first / last chunks
    "gen2_some": (2, [256, 64, 256], [(1, 1, free(1, lambda t: 0.3 * math.sin(2 * t))),
                                      (1, -1, {"Vy": lambda t: 0.1, "Sxy": lambda t: 0.0}),
                                      (2, 0, free(2)), (0, -1, {"Vx": lambda t: 0.05})], 0.9, "fused"),
}


@pytest.mark.parametrize("name", sorted(FACE_CASES))
def test_step_faces_matches_oracle(G, name):
    bs, sizes, conds, tau, path = FACE_CASES[name]
    b = face_body(3, bs, sizes, conds)
    random_state(b, seed=len(name) + sizes[2], ghosts=False)
    ctx = context_for(b)
    t = 0.0
    for step in range(3):
        for s in range(3):
            b.apply_border(s, t)
            b.stage(s, tau)
        ctx.step_faces(tau, faces_at(3, conds, t))
        assert ctx.last_path == path, f"{name}: ran {ctx.last_path}"
        assert_same_inner(ctx, b, f"faces {name} step {step}")
        t += tau


def test_step_faces_512_slab_headline_instance(G):
    """The benchmark kernel instance (bs 2, Z = ZT = 512, uniform axes) with free
    surfaces on every face, a thin slab of the 512^3 grid."""
    conds = [(0, 0, free(0)), (1, 0, free(1, lambda t: 0.1)), (2, 0, free(2))]
    b = face_body(3, 2, [4, 24, 512], conds)
    random_state(b, seed=512, ghosts=False)
    ctx = context_for(b)
    for step in range(2):
        for s in range(3):
            b.apply_border(s, 0.0)
            b.stage(s, 0.9)
        ctx.step_faces(0.9, faces_at(3, conds, 0.0))
        assert ctx.last_path == "fused"
        assert_same_inner(ctx, b, f"512 slab step {step}")


def test_step_faces_2d_and_1d(G):
    """gcmx_step_faces in 2-D and 1-D (per-stage path, device face fills)."""
    for D, sizes, conds in ((2, [15, 11], [(0, 0, {"Sxx": lambda t: 0.2, "Sxy": lambda t: 0.0}),
                                          (1, 1, {"Vy": lambda t: -0.1})]),
                            (1, [40], [(0, 0, {"Sxx": lambda t: 0.5})])):
        bcs = [O.BorderCondition(a, ("infinite",) if s == 0 else face_area(D, sizes, a, s), v)
               for a, s, v in conds]
        task = O.Task(D=D, border_size=2, h=[1.0] * D, cubics={0: (sizes, [0] * D)}, courant=0.9,
                      default_material=O.Material(4.0, 2.0, 1.0), number_of_snaps=1,
                      border_conditions={0: bcs})
        b = O.Engine(task).bodies[0]
        random_state(b, seed=D, ghosts=False)
        ctx = context_for(b)
        for step in range(3):
            for s in range(D):
                b.apply_border(s, 0.0)
                b.stage(s, 0.9)
            ctx.step_faces(0.9, faces_at(D, conds, 0.0))
            assert_same_inner(ctx, b, f"D={D} step {step}")


def test_step_faces_after_split_fills_keeps_parity(G):
    """A face filled in memory by an earlier per-stage step and disabled later keeps
    its stale ghosts, as in the reference: the library must not run the one-pass
    step then (it would read zeros there)."""
    conds = [(1, 0, free(1)), (2, 0, free(2))]
    b = face_body(3, 2, [6, 12, 20], conds)
    random_state(b, seed=5, ghosts=False)
    ctx = context_for(b)
    ctx.set_path(G.PATH_SPLIT)
    for s in range(3):
        b.apply_border(s, 0.0)
        b.stage(s, 0.9)
    ctx.step_faces(0.9, faces_at(3, conds, 0.0))
    assert ctx.last_path == "split"
    ctx.set_path(G.PATH_AUTO)
    only_z = [(2, 0, free(2))]  # the y faces drop out; their ghost rows keep old values
    b.border = [e for e in b.border if e[0] == 2]
    for s in range(3):
        b.apply_border(s, 0.0)
        b.stage(s, 0.9)
    ctx.step_faces(0.9, faces_at(3, only_z, 0.0))
    assert ctx.last_path == "split"
    assert_same(ctx, b, "stale y ghosts")


def test_border_nodes_apply_matches_oracle(G):
    """Device-resident node lists: uploaded once, applied per stage."""
    D, bs = 3, 2
    sizes = [7, 9, 8]
    conds = [O.BorderCondition(0, ("box", (-1, 1.5, -1), (100, 5.5, 100)),
                               {"Sxx": lambda t: 0.5, "Sxy": lambda t: -0.25}),
             O.BorderCondition(1, ("infinite",), {"PRESSURE": lambda t: 0.125}),
             O.BorderCondition(2, ("sphere", 4, (3, 4, 0)), {"Vz": lambda t: 0.3})]
    t = O.Task(D=D, border_size=bs, h=[1.0] * D, cubics={0: (sizes, [0] * D)}, courant=0.9,
               default_material=O.Material(4, 2, 1), number_of_snaps=1, border_conditions={0: conds})
    b = O.Engine(t).bodies[0]
    random_state(b, seed=9, ghosts=True)
    ctx = context_for(b)
    handles = [(d, ctx.border_nodes(d, -1, left), ctx.border_nodes(d, +1, right), vals)
               for d, left, right, vals in b.border]
    for rep in range(2):
        for direction in range(D):
            b.apply_border(direction, 0.1 * rep)
            for d, hl, hr, vals in handles:
                if d != direction:
                    continue
                qs = [QCODE[q] for q, _ in vals]
                vs = [f(0.1 * rep) for _, f in vals]
                ctx.border_apply(hl, qs, vs)
                ctx.border_apply(hr, qs, vs)
            assert_same(ctx, b, f"border nodes direction {direction} rep {rep}")
            b.stage(direction, 0.9)
            ctx.stage(direction, 0.9)
            assert_same(ctx, b, f"stage {direction} rep {rep}")


@pytest.fixture(scope="module")
def H():
    from gcm_amd import _gcm_host
    return _gcm_host


def run_both(H, s):
    oe = O.Engine(oracle_task(s))
    he = H.Engine(host_task(s))
    oe.run()
    he.run()
    assert he.steps == oe.steps_done
    return oe, he


def test_engine_free_surfaces_one_pass(H):
    """The cube task's free surfaces (launcher/main.cpp:209-220: FIXED_FORCE zero on
    every face) plus a time-dependent normal load on the top face, through
    Task -> Engine::run: whole-face conditions, so every step is one pass."""
    f = lambda t: -0.4 * math.exp(-(t - 1.0) ** 2)
    N = 16
    s = spec(3, 2, [1, 1, 1], {0: ([N, N + 2, N + 4], [0, 0, 0])}, 0.9, (4, 2, 1), snaps=6,
             quantities=[(("sphere", 4, (8, 9, 10)), "PRESSURE", 1.0)],
             borders={0: [(0, ("infinite",), {q: (lambda t: 0.0) for q in FREE[0]}),
                          (1, ("infinite",), {q: (lambda t: 0.0) for q in FREE[1]}),
                          (2, ("infinite",), {q: (lambda t: 0.0) for q in FREE[2]}),
                          (1, ("box", (-1e3, N + 0.5, -1e3), (1e3, N + 1.5, 1e3)),
                           {"Syy": f, "Sxy": lambda t: 0.0, "Syz": lambda t: 0.0})]})
    oe, he = run_both(H, s)
    assert he.last_path(0) == "fused"
    b = oe.bodies[0]
    got = b.inner_view(he.pde(0).reshape(b.pde.shape))
    want = b.inner_view(b.pde)
    assert np.array_equal(got, want), f"{int((got != want).sum())} inner values differ"


@pytest.mark.parametrize("maps", [True, False])
def test_engine_partial_face_uses_node_lists(H, monkeypatch, maps):
    """A condition covering part of a face (titan's cylinder, ndi.hpp:309-315):
    with face maps the one-pass step, with GCMX_NO_FACE_MAPS=1 the per-stage path
    with device-resident node lists; both bitwise == the oracle."""
    if not maps:
        monkeypatch.setenv("GCMX_NO_FACE_MAPS", "1")
    N = 12
    s = spec(3, 2, [1, 1, 1], {0: ([N, N, N], [0, 0, 0])}, 0.9, (4, 2, 1), snaps=4,
             quantities=[(("sphere", 3, (6, 6, 6)), "PRESSURE", 1.0)],
             borders={0: [(1, ("infinite",), {q: (lambda t: 0.0) for q in FREE[1]}),
                          (1, ("cylinder", 2.5, (6, -5, 6), (6, 20, 6)), {"Vy": lambda t: -0.3})]})
    oe, he = run_both(H, s)
    assert he.last_path(0) == ("fused" if maps else "split")
    got = he.pde(0)
    want = oe.bodies[0].pde.reshape(got.shape)
    if maps:  # the one-pass step never writes y/z face ghosts (oracle: scratch)
        got, want = got[2:-2, 2:-2, 2:-2], want[2:-2, 2:-2, 2:-2]
    assert np.array_equal(got, want), f"{int((got != want).sum())} values differ"


@pytest.mark.parametrize("layout", ["random", "layers"])
def test_step_faces_heterogeneous_one_pass(G, layout):
    """Per-node materials (k_step_tx2<..., FACES, HET>) with whole-face conditions:
    free surfaces, a time-dependent normal force on y+ and a velocity on x-; each
    node's stages use its own material (random ids, or two layers along x) ==
    the oracle's per-stage border fills and stages, inner nodes bitwise."""
    from tests.helpers import random_materials
    sizes = [8, 18, 64]
    conds = [(0, 0, free(0)), (1, 0, free(1)), (1, 1, free(1, lambda t: 0.3 * math.sin(2 * t))),
             (2, 0, free(2)), (0, -1, {"Vx": lambda t: 0.05})]
    bcs = []
    for axis, side, vals in conds:
        area = ("infinite",) if side == 0 else face_area(3, sizes, axis, side)
        bcs.append(O.BorderCondition(axis, area, vals))
    mats = [O.Material(4.0, 2.0, 1.0), O.Material(1.0, 2.0, 0.8)]
    t_ = O.Task(D=3, border_size=2, h=[1.0] * 3, cubics={0: (sizes, [0, 0, 0])}, courant=0.9,
                default_material=mats[0], inhomogeneities=[(("infinite",), mats[1])], number_of_snaps=1,
                border_conditions={0: bcs})
    b = O.Engine(t_).bodies[0]
    if layout == "random":
        random_materials(b, seed=8)
    else:
        its = b.inner_indices()
        b.mat_id[b.flat_index(its)] = np.where(its[:, 0] < sizes[0] // 2, 0, 1).astype(np.uint8)
    random_state(b, seed=9, ghosts=False)
    ctx = context_for(b)
    tau = 0.9 / math.sqrt(3.0)  # Courant 0.9 on the faster material (floor(q) = 0)
    t = 0.0
    for step in range(3):
        for s in range(3):
            b.apply_border(s, t)
            b.stage(s, tau)
        ctx.step_faces(tau, faces_at(3, conds, t))
        assert ctx.last_path == "fused"
        assert_same_inner(ctx, b, f"faces HET {layout} step {step}")
        t += tau


# ---- partial faces: per-node face maps (gcmx_face_map) -----------------------

def face_maps(b, sizes):
    """Per face the LAST condition covering each face node (the oracle body's
    border list is in the reference's application order), 255 where none."""
    maps = [None] * 6
    for k, (d, left, right, vals) in enumerate(b.border):
        other = [a for a in range(3) if a != d]
        for side, nodes in ((0, left), (1, right)):
            if len(nodes) == 0:
                continue
            f = 2 * d + side
            if maps[f] is None:
                maps[f] = np.full(sizes[other[0]] * sizes[other[1]], 255, dtype=np.uint8)
            maps[f][nodes[:, other[0]] * sizes[other[1]] + nodes[:, other[1]]] = k
    return maps


def conditions_at(b, time):
    return [[(QCODE[q], f(time)) for q, f in vals] for (_, _, _, vals) in b.border]


PARTIAL_CASES = {
    # half of y- free, a sphere cap of y+ with a normal force, z faces free with a
    # later override on part of z+, part of x- with a velocity
    "mixed": (2, [10, 24, 64], [
        (1, -1, ("box", (-1, -1, -1), (4.5, 1, 100)), free(1)),
        (1, 1, ("sphere", 6.0, (5, 23, 30)), free(1, lambda t: 0.2 + 0.1 * t)),
        (2, 0, ("infinite",), free(2)),
        (2, 1, ("box", (3.5, 5.5, -100), (100, 15.5, 100)), {"Vz": lambda t: -0.1, "Sxz": lambda t: 0.0}),
        (0, -1, ("box", (-100, -1, 20.5), (100, 12.5, 100)), {"Vx": lambda t: 0.05}),
    ], 0.9, "fused"),
    # Z with idle lanes and odd X, overlapping conditions on a y face
    "idle_lanes": (2, [9, 20, 70], [
        (1, 0, ("box", (-1, -100, -1), (5.5, 100, 40.5)), free(1)),
        (1, 0, ("box", (2.5, -100, 20.5), (100, 100, 100)), {"Vy": lambda t: 0.1}),
        (2, -1, ("box", (-1, 3.5, -100), (100, 11.5, 100)), free(2)),
    ], 0.9, "fused"),
    # PRESSURE on part of an x face: filled in memory, still one pass
    "pressure_x": (2, [8, 16, 64], [
        (0, 1, ("box", (-100, -1, -1), (100, 8.5, 30.5)), {"PRESSURE": lambda t: 0.25}),
        (1, -1, ("box", (-1, -100, 10.5), (100, 100, 50.5)), free(1)),
    ], 0.9, "fused"),
    # PRESSURE on part of a z face: its trace needs node-only components -> per stage
    "pressure_z": (2, [6, 14, 40], [
        (2, 1, ("box", (-1, 3.5, -100), (100, 9.5, 100)), {"PRESSURE": lambda t: -0.1}),
        (1, 0, ("box", (2.5, -100, -1), (100, 100, 100)), free(1)),
    ], 0.9, "split"),
    "bs1": (1, [7, 12, 64], [
        (1, 0, ("box", (-1, -100, 10.5), (100, 100, 40.5)), free(1)),
        (2, 0, ("box", (2.5, 2.5, -100), (100, 100, 100)), free(2)),
    ], 0.9, "fused"),
    # rows of 1024 (z split): partial y faces across the cut columns (z 508-515)
    # and on both parts, a partial z+ face in the last part
    "z1024": (2, [6, 10, 1024], [
        (1, -1, ("box", (-1, -1, 300.5), (100, 1, 700.5)), free(1)),
        (1, 1, ("box", (2.5, 8, -1), (100, 100, 511.5)), free(1, lambda t: 0.2 + 0.1 * t)),
        (2, 1, ("box", (-1, 3.5, -100), (100, 7.5, 2000)), {"Vz": lambda t: -0.1}),
    ], 0.9, "fused"),
}


def partial_body(bs, sizes, conds, materials=((4.0, 2.0, 1.0),)):
    bcs = []
    for axis, side, area, vals in conds:
        if side != 0:  # restrict the area to one face: intersect with the face slab
            fa = face_area(3, sizes, axis, side)
            lo = [max(a, b) for a, b in zip(fa[1], area[1])] if area[0] == "box" else None
            if area[0] == "box":
                hi = [min(a, b) for a, b in zip(fa[2], area[2])]
                area = ("box", tuple(lo), tuple(hi))
            elif area[0] == "sphere":  # a sphere whose centre sits on the face touches only it here
                pass
        bcs.append(O.BorderCondition(axis, area, vals))
    mats = [O.Material(*m) for m in materials]
    t = O.Task(D=3, border_size=bs, h=[1.0] * 3, cubics={0: (list(sizes), [0] * 3)}, courant=0.9,
               default_material=mats[0], inhomogeneities=[(("infinite",), m) for m in mats[1:]],
               number_of_snaps=1, border_conditions={0: bcs})
    return O.Engine(t).bodies[0]


@pytest.mark.parametrize("name", sorted(PARTIAL_CASES))
@pytest.mark.parametrize("fp", ["exact", "fma"])
def test_step_face_map_matches_oracle(G, name, fp):
    """VERDICT r3 missing 4: PARTIAL faces (a condition's area covers part of a
    face; the titan preset's cylinder, ndi.hpp:309-315) in the one-pass step --
    every face node's ghosts from its own last condition, zero where none --
    against the oracle's BorderConditions::apply + stage sequence: bitwise in the
    exact build, within 1e-10 relative L2 in the FMA build."""
    bs, sizes, conds, tau, path = PARTIAL_CASES[name]
    b = partial_body(bs, sizes, conds)
    random_state(b, seed=len(name) + sizes[2], ghosts=False)
    ctx = context_for(b)
    if fp == "fma":
        ctx.fp_mode = G.FP_FMA
    fmap = ctx.face_map(face_maps(b, sizes))
    t = 0.0
    for step in range(3):
        for s in range(3):
            b.apply_border(s, t)
            b.stage(s, tau)
        ctx.step_face_map(tau, fmap, conditions_at(b, t))
        assert ctx.last_path == path, f"{name}: ran {ctx.last_path}"
        if fp == "exact":
            assert_same_inner(ctx, b, f"partial {name} step {step}")
        else:
            got = b.inner_view(ctx.download().reshape(b.pde.shape))
            want = b.inner_view(b.pde)
            r = float(np.linalg.norm(got - want)) / float(np.linalg.norm(want))
            assert r <= 1e-10, f"partial {name} step {step}: {r}"
        t += tau
    fmap.close()
    ctx.close()


@pytest.mark.parametrize("name", ["mixed", "bs1"])
def test_step_face_map_heterogeneous_one_pass(G, name):
    """Partial faces AND per-node materials (random ids, two materials in most
    lane pairs) in one one-pass launch (k_step_tx2<..., FACES, HET>): bitwise ==
    the oracle's BorderConditions::apply + stage sequence with each node's own
    matrices."""
    from tests.helpers import random_materials
    bs, sizes, conds, _, path = PARTIAL_CASES[name]
    b = partial_body(bs, sizes, conds, materials=((4.0, 2.0, 1.0), (1.0, 2.0, 0.8)))
    random_materials(b, seed=3)
    random_state(b, seed=11, ghosts=False)
    tau = 0.9 / np.sqrt(3.6)  # Courant 0.9 on the faster material: floor(q) = 0 for both
    ctx = context_for(b)
    ctx.profile(True)
    fmap = ctx.face_map(face_maps(b, sizes))
    t = 0.0
    for step in range(3):
        for s in range(3):
            b.apply_border(s, t)
            b.stage(s, tau)
        ctx.step_face_map(tau, fmap, conditions_at(b, t))
        assert ctx.last_path == path == "fused"
        assert_same_inner(ctx, b, f"partial HET {name} step {step}")
        t += tau
    k = ctx.profile_read()
    assert "HET" in k["fused_xyz"]["kernel"] and ", FACES," in k["fused_xyz"]["kernel"], k
    fmap.close()
    ctx.close()


def test_face_map_refuses_bad_maps(G):
    b = partial_body(2, [6, 12, 64], PARTIAL_CASES["bs1"][2])
    ctx = context_for(b)
    bad = [None, None, np.full(6 * 64, 9, dtype=np.uint8), None, None, None]  # index >= 8
    with pytest.raises(G.GcmxError):
        ctx.face_map(bad)
    fmap = ctx.face_map([None, None, np.zeros(6 * 64, dtype=np.uint8), None, None, None])
    with pytest.raises(G.GcmxError):  # the map names condition 0, none given
        ctx.step_face_map(0.9, fmap, [])
    fmap.close()
    ctx.close()


def test_context_close_closes_its_face_maps_and_node_lists(G):
    """gcmx_face_map_destroy / gcmx_border_nodes_destroy read their
    context (device, stream), so a FaceMap or BorderNodes outliving an explicit
    Context.close() must not call them afterwards.  The context closes its
    children first; their later close() (or collection) is then a no-op."""
    b = partial_body(2, [6, 12, 64], PARTIAL_CASES["bs1"][2])
    ctx = context_for(b)
    fmap = ctx.face_map([None, None, np.zeros(6 * 64, dtype=np.uint8), None, None, None])
    nodes = ctx.border_nodes(1, -1, np.array([[0, 0, 0], [1, 0, 3]], dtype=np.int32))
    ctx.close()
    assert not fmap.ptr.value and not nodes.ptr.value  # closed with their context
    fmap.close()
    nodes.close()
    del fmap, nodes


def test_engine_partial_faces_one_pass(G):
    """A titan-like body through the C++ engine: border conditions whose areas
    cover parts of faces -> HipBorderConditions builds the per-node face map and
    the engine runs gcmx_step_face_map (one pass); bitwise == the oracle engine."""
    from gcm_amd import _gcm_host as H
    s = spec(3, 2, [1, 1, 1], {0: ([10, 20, 64], [0, 0, 0])}, 0.9, (4, 2, 1), snaps=4,
             quantities=[(("sphere", 5.0, (5, 10, 32)), "PRESSURE", 10.0)],
             borders={0: [(1, ("box", (-1, -1, -1), (4.5, 0.5, 100)),
                           {"Syy": lambda t: 0.0, "Sxy": lambda t: 0.0, "Syz": lambda t: 0.0}),
                          (2, ("sphere", 8.0, (5, 10, 63)),
                           {"Szz": lambda t: -0.2, "Sxz": lambda t: 0.0, "Syz": lambda t: 0.0}),
                          (0, ("box", (-1, -1, -1), (0.5, 9.5, 100)), {"Vx": lambda t: 0.01})]})
    he = H.Engine(host_task(s))
    he.run()
    assert he.last_path(0) == "fused"
    oe = O.Engine(oracle_task(s))
    oe.run()
    assert he.steps == oe.steps_done
    got = he.pde(0)
    want = oe.bodies[0].pde.reshape(got.shape)
    gi, wi = got[2:-2, 2:-2, 2:-2], want[2:-2, 2:-2, 2:-2]
    assert np.array_equal(gi, wi), int((gi != wi).sum())
