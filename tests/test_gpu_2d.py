"""The one-pass 2-D step (k_step2d) against the oracle, bitwise.

gcmx_step on a 2-D context with one material and untouched ghosts runs the X
and Y stages of Engine::nextTimeStep (Engine.cpp:90-121) in one kernel; each
stage's arithmetic is k_stage_generic's (GridCharacteristicMethod.hpp:42-52),
so the result is IEEE-equal to two oracle stages.  The cases cover borderSize
1..5, feet more than one cell away (Courant 2.5, TestEngine's bs = 5 grids), a
single column / row, grids narrower than one 64-lane block, and grids needing
several 256-lane column blocks (whose halo columns each block forms itself).
"""
import math

import numpy as np
import pytest

from tests.helpers import assert_same, context_for, oracle_body, random_state

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G():
    import gcm_amd
    gcm_amd.lib()
    return gcm_amd


CASES = [
    (1, [9, 13], 0.9), (2, [21, 70], 0.9), (2, [100, 50], 0.9), (3, [17, 5], 0.9),
    (5, [20, 40], 0.9), (1, [1, 300], 0.9), (1, [300, 1], 0.9), (2, [2, 300], 0.9), (2, [33, 61], 0.9),
    (2, [7, 600], 0.9), (4, [40, 509], 0.9), (1, [130, 253], 0.9),
    (3, [12, 30], 2.5), (5, [9, 270], 4.5),
]


@pytest.mark.parametrize("bs,sizes,courant", CASES)
def test_step2d_matches_oracle(G, bs, sizes, courant):
    b = oracle_body(2, bs, sizes, h=[1.0, 0.5])
    random_state(b, seed=bs * 100 + sizes[0] + sizes[1], ghosts=False)
    ctx = context_for(b)
    assert ctx.effective_path == "fused"
    tau = courant * 0.5 / 1.0  # Courant number on the smaller h (c1 = 1 for (4, 2, 1))
    for step in range(3):
        for s in range(2):
            b.stage(s, tau)
        ctx.step(tau)
        assert ctx.last_path == "fused"
        assert_same(ctx, b, f"2-D step bs={bs} sizes={sizes} courant={courant} step {step}")
    ctx.close()


def test_step2d_equals_generic_stages_large(G):
    """A grid the oracle would take long over (2 000 x 3 000, 12 column blocks):
    the one-pass step equals the two generic stage kernels, bitwise."""
    import gcm_amd
    X, Y = 2000, 3000
    ctxs = []
    for path in (G.PATH_AUTO, G.PATH_GENERIC):
        c = gcm_amd.Context(2, 2, [X, Y], h=[1.0, 0.5])
        b = oracle_body(2, 2, [4, 4], h=[1.0, 0.5])  # tables only
        U = np.stack([t[0] for t in b.tables]); U1 = np.stack([t[1] for t in b.tables])
        L = np.stack([t[2] for t in b.tables])
        c.set_materials(U, U1, L)
        c.set_path(path)
        c.fill_random([X, Y], 0x2D)
        ctxs.append(c)
    assert ctxs[0].effective_path == "fused" and ctxs[1].effective_path == "generic"
    for _ in range(4):
        for c in ctxs:
            c.step(0.45)
    a, g = ctxs[0].download(), ctxs[1].download()
    assert np.array_equal(a, g)
    assert np.abs(a).sum() > 0
    for c in ctxs:
        c.close()


def test_step2d_ode_equals_generic(G):
    """gcmx_step_ode on the 2-D step: the one-pass step, then the Maxwell ODE pass."""
    b = oracle_body(2, 2, [40, 90], h=[1.0, 0.5])
    random_state(b, seed=9, ghosts=False)
    fused, generic = context_for(b), context_for(b, path=G.PATH_GENERIC)
    assert fused.effective_path == "fused"
    for _ in range(3):
        fused.step_ode(0.45, [2.0])
        generic.step_ode(0.45, [2.0])
    assert np.array_equal(fused.download(), generic.download())
    fused.close()
    generic.close()


def test_step2d_not_taken_with_ghosts_or_materials(G):
    """Non-zero ghosts (the two layers' ghosts would differ) or per-node materials
    keep the per-stage generic path, which equals the oracle as before."""
    b = oracle_body(2, 2, [15, 20], h=[1.0, 0.5])
    random_state(b, seed=4, ghosts=True)
    ctx = context_for(b)
    assert ctx.effective_path == "generic"
    for s in range(2):
        b.stage(s, 0.45)
    ctx.step(0.45)
    assert ctx.last_path == "generic"
    assert_same(ctx, b, "2-D step with ghosts")
    ctx.close()
    m = oracle_body(2, 2, [15, 20], h=[1.0, 0.5], materials=((4.0, 2.0, 1.0), (1.0, 2.0, 0.8)))
    random_state(m, seed=5, ghosts=False)
    ctx = context_for(m)
    assert ctx.effective_path == "generic"
    ctx.close()


def _kernel_of_one_step(ctx, tau):
    ctx.profile(True)
    ctx.profile_reset()
    ctx.step(tau)
    ctx.sync()
    p = ctx.profile_read()
    ctx.profile(False)
    return p["step2d"]


@pytest.mark.parametrize("bs,courant,kernel", [(2, 0.9, "k_step2d_iso<2, 256, KF0>"),
                                               (3, 2.5, "k_step2d_iso<3, 256, !KF0>"),
                                               (4, 0.9, "k_step2d<4, 256>")])
def test_step2d_profile_bucket(G, bs, courant, kernel):
    """The step's profile bucket names the instance (the isotropic kernel up to
    borderSize 3, the table kernel above) and prices 80 B per node."""
    b = oracle_body(2, bs, [64, 500], h=[1.0, 0.5])
    random_state(b, seed=3, ghosts=False)
    ctx = context_for(b)
    p = _kernel_of_one_step(ctx, courant * 0.5)
    assert p["kernel"] == kernel
    assert p["bytes_per_launch"] == 80 * 64 * 500
    ctx.close()


@pytest.mark.parametrize("bs", [1, 2, 3])
def test_step2d_table_kernel_for_other_matrices(G, bs):
    """Matrices off the isotropic structure (one structural zero of U made
    non-zero) run the table kernel, which equals two oracle stages bitwise."""
    b = oracle_body(2, bs, [30, 300], h=[1.0, 0.5])
    for t in b.tables:
        t[0][0][0, 4] = 1e-3  # U of axis 0, row 0, sigma_yy: zero in ElasticModel<2>
    random_state(b, seed=8 + bs, ghosts=False)
    ctx = context_for(b)
    assert ctx.effective_path == "fused"
    tau = 0.45
    for step in range(2):
        for s in range(2):
            b.stage(s, tau)
        if step == 0:
            assert _kernel_of_one_step(ctx, tau)["kernel"].startswith("k_step2d<")
        else:
            ctx.step(tau)
        assert_same(ctx, b, f"table kernel bs={bs} step {step}")
    ctx.close()


# ------------------------------------------------------------- y/x faces --

QCODE = {"Vx": 2, "Vy": 3, "Sxx": 5, "Sxy": 6, "Syy": 8, "PRESSURE": 12}
FREE2 = {0: ("Sxx", "Sxy"), 1: ("Syy", "Sxy")}  # free surface of a 2-D face (ndi.hpp:30-55)


def free2(axis, normal=lambda t: 0.0):
    q = FREE2[axis]
    return {q[0]: normal, q[1]: lambda t: 0.0}


def face_body2(bs, sizes, conditions):
    """conditions: (axis, side or 0 for both faces, {quantity: f(t)}), h = 1."""
    from oracle import oracle as O
    bcs = []
    for axis, side, vals in conditions:
        if side == 0:
            area = ("infinite",)
        else:
            lo, hi = [-1e3] * 3, [1e3] * 3
            c = 0.0 if side < 0 else float(sizes[axis] - 1)
            lo[axis], hi[axis] = c - 0.5, c + 0.5
            area = ("box", tuple(lo), tuple(hi))
        bcs.append(O.BorderCondition(axis, area, vals))
    t = O.Task(D=2, border_size=bs, h=[1.0, 1.0], cubics={0: (list(sizes), [0, 0])}, courant=0.9,
               default_material=O.Material(4.0, 2.0, 1.0), number_of_snaps=1, border_conditions={0: bcs})
    return O.Engine(t).bodies[0]


def faces_at2(conditions, time):
    from oracle import oracle as O
    faces = [None] * 4
    for axis, side, vals in conditions:
        lst = sorted(vals.items(), key=lambda kv: O.QUANTITY_ORDER.index(kv[0]))
        entry = [(QCODE[q], f(time)) for q, f in lst]
        for s in ((0, 1) if side == 0 else ((0,) if side < 0 else (1,))):
            faces[2 * axis + s] = entry
    return faces


FACE2_CASES = {
    "free_all": (2, [30, 70], [(0, 0, free2(0)), (1, 0, free2(1))], 0.9, "fused"),
    "some_faces": (2, [25, 40], [(1, 1, free2(1, lambda t: 0.3 * math.sin(2 * t))),
                                 (0, -1, {"Vx": lambda t: 0.05})], 0.9, "fused"),
    "override": (2, [12, 22], [(1, 0, free2(1)), (1, -1, {"Vy": lambda t: 0.1, "Sxy": lambda t: 0.0})],
                 0.9, "fused"),
    "bs1_narrow": (1, [9, 2], [(0, 0, free2(0)), (1, 0, free2(1))], 0.9, "fused"),
    "bs3_courant25": (3, [14, 33], [(0, 0, free2(0)), (1, 0, free2(1, lambda t: -0.2))], 2.5, "fused"),
    "column_blocks": (2, [10, 600], [(1, 0, free2(1)), (0, 1, free2(0))], 0.9, "fused"),
    "pressure_y": (2, [8, 20], [(1, -1, {"PRESSURE": lambda t: 0.25}), (0, 0, free2(0))], 0.9, "generic"),
    "pressure_x": (2, [8, 20], [(0, 1, {"PRESSURE": lambda t: 0.25}), (1, 0, free2(1))], 0.9, "fused"),
}


@pytest.mark.parametrize("name", sorted(FACE2_CASES))
def test_step2d_faces_matches_oracle(G, name):
    """gcmx_step_faces in 2-D: x faces filled in memory, the y faces' ghost
    columns formed in the one pass from the mirrored columns; inner nodes equal
    the reference's apply_border + stage sequence bitwise (the ghosts of the
    intermediate layer exist only on the chip)."""
    from tests.helpers import assert_same_inner
    bs, sizes, conds, courant, path = FACE2_CASES[name]
    b = face_body2(bs, sizes, conds)
    random_state(b, seed=len(name) + sizes[1], ghosts=False)
    ctx = context_for(b)
    tau, t = courant, 0.0  # h = 1, c1 = 1
    for step in range(3):
        for s in range(2):
            b.apply_border(s, t)
            b.stage(s, tau)
        ctx.step_faces(tau, faces_at2(conds, t))
        assert ctx.last_path == path, f"{name}: ran {ctx.last_path}"
        assert_same_inner(ctx, b, f"2-D faces {name} step {step}")
        t += tau
    ctx.close()


def test_step2d_faces_kernel_and_plain_step_after(G):
    """The faces step names its FACES instance; a plain gcmx_step after it (x face
    ghosts written in memory, not refreshed) takes the per-stage path."""
    conds = [(0, 0, free2(0)), (1, 0, free2(1))]
    b = face_body2(2, [16, 300], conds)
    random_state(b, seed=2, ghosts=False)
    ctx = context_for(b)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.step_faces(0.9, faces_at2(conds, 0.0))
    ctx.sync()
    assert ctx.profile_read()["step2d"]["kernel"] == "k_step2d_iso<2, 256, KF0, FACES>"
    ctx.profile(False)
    assert ctx.effective_path == "generic"
    ctx.close()
