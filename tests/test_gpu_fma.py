"""The product default of the one-pass step: GCMX_FP_FMA (kernels_xyz.hip
compiled with multiply-adds contracted, gcmx_set_fp_mode).  The north star asks
for fields within 1e-10 relative L2 of the reference CPU solver on identical
inputs; these tests hold the FMA build to that tolerance against the oracle
(which is bitwise equal to the reference path, tests/test_oracle.py) on every
specialisation of k_step_tx2 / k_fused_xyz the product launches, and check that
its multi-GPU schedules are bitwise equal to the undivided FMA step (the same
kernel code on plane ranges).  The rest of the suite runs the exact build
(GCMX_FP_EXACT, conftest.py) and compares bitwise.

Tolerance: relative L2 over all inner nodes and components,
||gpu - oracle||_2 / ||oracle||_2 <= 1e-10 after every step (measured values are
~1e-16; the assertion message prints them)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import context_for, oracle_body, random_materials, random_state
from tests.test_gpu_faces import FACE_CASES, face_body, faces_at

pytestmark = pytest.mark.gpu

TOL = 1e-10  # north star: fields within 1e-10 relative L2 of the reference


@pytest.fixture(scope="module")
def G():
    import gcm_amd
    gcm_amd.lib()
    return gcm_amd


def rel_l2(got, want):
    n = float(np.linalg.norm(want))
    return float(np.linalg.norm(got - want)) / (n if n > 0 else 1.0)


def check(ctx, b, what):
    got = b.inner_view(ctx.download().reshape(b.pde.shape))
    want = b.inner_view(b.pde)
    r = rel_l2(got, want)
    assert r <= TOL, f"{what}: relative L2 {r:.3e} > {TOL}"
    return r


def fma_ctx(G, b):
    ctx = context_for(b)
    ctx.fp_mode = G.FP_FMA
    assert ctx.fp_mode == G.FP_FMA
    return ctx


def test_fp_mode_api(G):
    """Default of a new context is FMA unless GCMX_FP=exact (the suite sets it);
    unknown modes are refused."""
    b = oracle_body(3, 2, [4, 8, 64])
    ctx = context_for(b)
    assert ctx.fp_mode == G.FP_EXACT  # conftest: GCMX_FP=exact
    ctx.fp_mode = G.FP_FMA
    assert ctx.fp_mode == G.FP_FMA
    with pytest.raises(G.GcmxError):
        ctx.fp_mode = 7
    ctx.close()


@pytest.mark.parametrize("bs,sizes", [(2, [6, 24, 512]), (2, [5, 20, 256]), (2, [7, 9, 128]),
                                      (2, [12, 10, 70]), (1, [4, 3, 64]), (3, [9, 7, 100]),
                                      (2, [4, 12, 1024])])
def test_fma_step_within_tolerance(G, bs, sizes):
    """k_step_tx2 (bs <= 2, Z <= 512; [6, 24, 512] is the 512^3 bench instance,
    Z = 70 has idle lanes) and k_fused_xyz (bs 3, Z > 512) in the FMA build: 5
    steps against the oracle within the tolerance, and not bitwise equal to the
    exact build (the contracted code really runs)."""
    b = oracle_body(3, bs, sizes)
    random_state(b, seed=sum(sizes), ghosts=False)
    ctx = fma_ctx(G, b)
    ex = context_for(b)
    assert ctx.effective_path == "fused"
    worst = 0.0
    for step in range(5):
        for s in range(3):
            b.stage(s, 0.9)
        ctx.step(0.9)
        ex.step(0.9)
        worst = max(worst, check(ctx, b, f"FMA bs={bs} sizes={sizes} step {step}"))
    assert np.array_equal(ex.download(), b.pde)  # the exact build stays bitwise
    assert not np.array_equal(ctx.download(), ex.download())
    for c in (ctx, ex):
        c.close()


def test_fma_large_courant_within_tolerance(G):
    """Courant 1.5 (floor(q) = 1 on the fast waves: the instances without shared
    x differences) in the FMA build."""
    b = oracle_body(3, 2, [8, 16, 64])
    random_state(b, seed=11, ghosts=False)
    ctx = fma_ctx(G, b)
    for step in range(3):
        for s in range(3):
            b.stage(s, 1.5)
        ctx.step(1.5)
        check(ctx, b, f"FMA Courant 1.5 step {step}")
    ctx.close()


@pytest.mark.parametrize("name", ["free_all", "some_faces", "bs1", "courant15", "pressure_x"])
def test_fma_step_faces_within_tolerance(G, name):
    """Whole-face border conditions inside the FMA one-pass step (k_step_tx2<FACES>)."""
    bs, sizes, conds, tau, path = FACE_CASES[name]
    b = face_body(3, bs, sizes, conds)
    random_state(b, seed=len(name) + sizes[2], ghosts=False)
    ctx = fma_ctx(G, b)
    t = 0.0
    for step in range(3):
        for s in range(3):
            b.apply_border(s, t)
            b.stage(s, tau)
        ctx.step_faces(tau, faces_at(3, conds, t))
        assert ctx.last_path == path
        check(ctx, b, f"FMA faces {name} step {step}")
        t += tau
    ctx.close()


@pytest.mark.parametrize("sizes,layout", [([6, 20, 64], "random"), ([6, 24, 512], "layers")])
def test_fma_heterogeneous_within_tolerance(G, sizes, layout):
    """Per-node materials (k_step_tx2<..., HET>) in the FMA build."""
    mats = ((4.0, 2.0, 1.0), (1.0, 2.0, 0.8), (2.5, 0.0, 3.0))
    b = oracle_body(3, 2, sizes, materials=mats, courant=0.9)
    if layout == "random":
        random_materials(b, seed=5)
    else:
        its = b.inner_indices()
        b.mat_id[b.flat_index(its)] = np.where(its[:, 0] < sizes[0] // 2, 0, 1).astype(np.uint8)
    random_state(b, seed=6, ghosts=False)
    ctx = fma_ctx(G, b)
    tau = 0.9 / np.sqrt((3.0 + 6.0) / 2.5)
    for step in range(3):
        for s in range(3):
            b.stage(s, tau)
        ctx.step(tau)
        assert ctx.last_path == "fused"
        check(ctx, b, f"FMA HET {layout} step {step}")
    ctx.close()


def test_fma_anchor_pressure_sphere(G):
    """The survey's sanity anchor (3-D N = 32, 5 steps, pressure sphere p = 10):
    the FMA build's sums within the tolerance of the reference's
    -63401.220461788325 and 225405.1366274695."""
    N = 32
    t = O.Task(D=3, border_size=2, h=[1, 1, 1], cubics={0: ([N] * 3, [0] * 3)}, courant=0.9,
               default_material=O.Material(4, 2, 1), number_of_snaps=5,
               ic_quantities=[(("sphere", N / 4, (N / 2,) * 3), "PRESSURE", 10.0)])
    b = O.Engine(t).bodies[0]
    ctx = fma_ctx(G, b)
    assert ctx.effective_path == "fused"
    for _ in range(5):
        ctx.step(0.9)
    got = b.inner_view(ctx.download().reshape(b.pde.shape))
    ctx.close()
    s, s2 = float(np.sum(got)), float(np.sum(got * got))
    assert abs(s - -63401.220461788325) <= TOL * 63401.220461788325, s
    assert abs(s2 - 225405.1366274695) <= TOL * 225405.1366274695, s2


@pytest.mark.parametrize("sched", ["bfirst", "xslab", "single"])
@pytest.mark.parametrize("xs", [[8, 6, 10], [9, 6, 7], [7, 5, 9, 3], [5, 8, 3]])
def test_fma_slab_group_equals_whole_bitwise(G, sched, xs):
    """The multi-GPU schedules in the FMA build (in-process group of X slabs,
    boundary-first / X-slab / one launch) within the tolerance of the oracle,
    and bitwise equal to the undivided FMA step for ANY split: k_step_tx2
    computes x planes in pairs whose two nodes take differently contracted
    instruction sequences, and the pairs are global ((2k, 2k+1) in the global
    x index), so a slab starting at an odd plane begins with a half pair and
    every node keeps its pair position (TestEngine.cpp:27-87 / TestMPI.cpp:146-150:
    split == unsplit, bitwise)."""
    import gcm_amd
    from gcm_amd.host import isotropic_elastic_matrices
    Y, Z, seed = 20, 64, 0x5EED
    Xg = sum(xs)
    U, U1, L = isotropic_elastic_matrices(3, 4, 2, 1)
    sc = {"xslab": G.SCHED_XSLAB, "bfirst": G.SCHED_BFIRST, "single": G.SCHED_SINGLE}[sched]
    slabs, x0 = [], 0
    for X in xs:
        c = gcm_amd.Context(3, 2, [X, Y, Z], start=[x0, 0, 0])
        c.set_materials(U[None], U1[None], L[None])
        c.fp_mode = G.FP_FMA
        c.fill_random([Xg, Y, Z], seed)
        c.set_schedule(sc)
        slabs.append(c)
        x0 += X
    G.comm_init_local(slabs)
    w = gcm_amd.Context(3, 2, [Xg, Y, Z])
    w.set_materials(U[None], U1[None], L[None])
    w.fp_mode = G.FP_FMA
    w.fill_random([Xg, Y, Z], seed)
    steps = 3
    G.local_group_steps(slabs, 0.9, steps)
    for _ in range(steps):
        w.step(0.9)
    inner = lambda c: c.download().reshape(tuple(s + 4 for s in c.sizes) + (9,))[2:-2, 2:-2, 2:-2]
    got = np.concatenate([inner(c) for c in slabs], axis=0)
    assert np.array_equal(got, inner(w)), rel_l2(got, inner(w))
    b = oracle_body(3, 2, [Xg, Y, Z])
    O.fill_random(b, [Xg, Y, Z], seed)
    for _ in range(steps):
        for s in range(3):
            b.stage(s, 0.9)
    r = rel_l2(got, b.inner_view())
    assert r <= TOL, r
    for c in slabs + [w]:
        c.close()


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_fma_full_size_512_within_tolerance_of_exact(G):
    """512^3, the bench configuration: one step of the FMA build within the
    tolerance of the exact build (bitwise equal to the oracle at this size,
    test_gpu_parity.py::test_full_size_512_step_matches_oracle)."""
    import gcm_amd
    from gcm_amd.host import isotropic_elastic_matrices
    N, seed = 512, 0x5EED
    U, U1, L = isotropic_elastic_matrices(3, 4, 2, 1)
    outs = {}
    for mode in (G.FP_FMA, G.FP_EXACT):
        c = gcm_amd.Context(3, 2, [N, N, N])
        c.set_materials(U[None], U1[None], L[None])
        c.fp_mode = mode
        c.fill_random([N, N, N], seed)
        c.step(0.9)
        outs[mode] = c.download()
        c.close()
    r = rel_l2(outs[G.FP_FMA], outs[G.FP_EXACT])
    assert 0 < r <= TOL, r


def _xbodies(widths, cx=None):
    """3-D bodies stacked along x with the given widths (contacts along the
    stage-0 axis only: the engine's one-pass path), pressure sphere across them
    centred at global x = cx (default: 1.5 left of the first contact)."""
    from tests.taskspec import spec
    Y, Z = 20, 64
    cubics, x0 = {}, 0
    for i, w in enumerate(widths):
        cubics[i] = ([w, Y, Z], [x0, 0, 0])
        x0 += w
    return spec(3, 2, [1, 1, 1], cubics, 0.9, (4, 2, 1), snaps=6,
                quantities=[(("sphere", 6.0, (widths[0] - 1.5 if cx is None else cx, Y / 2, Z / 2)),
                                "PRESSURE", 10.0)])


@pytest.mark.parametrize("widths", [[12, 12], [7, 5, 12], [9, 8, 7]])
def test_fma_engine_xbodies_equal_one_body(G, monkeypatch, widths):
    """The FMA build through the C++ engine (GCMX_FP unset: the product default)
    with bodies along x of ODD widths, i.e. bodies starting at odd global planes:
    every body's one-pass step pairs planes globally, so the bodies together are
    bitwise equal to one body (TestEngine.cpp:27-87's split == unsplit), and
    within the tolerance of the oracle."""
    from gcm_amd import _gcm_host as H
    from tests.taskspec import host_task, oracle_task
    monkeypatch.setenv("GCMX_FP", "fma")
    monkeypatch.setenv("GCMX_NO_STACKS", "1")  # separate bodies: the global pairing is what is tested
    split = H.Engine(host_task(_xbodies(widths)))
    split.run()
    assert all(split.last_path(i) == "fused" for i in range(len(widths)))
    one = H.Engine(host_task(_xbodies([sum(widths)], cx=widths[0] - 1.5)))
    one.run()
    parts = [split.pde(i)[2:-2, 2:-2, 2:-2] for i in range(len(widths))]
    whole = one.pde(0)[2:-2, 2:-2, 2:-2]
    got = np.concatenate(parts, axis=0)
    assert np.any(whole != 0)
    assert np.array_equal(got, whole), rel_l2(got, whole)
    oe = O.Engine(oracle_task(_xbodies(widths)))
    oe.run()
    want = np.concatenate([b.pde.reshape(split.pde(b.id).shape)[2:-2, 2:-2, 2:-2] for b in oe.bodies], axis=0)
    assert rel_l2(got, want) <= TOL
    # the exact build would match the oracle bitwise; the FMA one really ran
    assert not np.array_equal(got, want)


@pytest.mark.parametrize("faces", [False, True])
def test_fma_step_ode_fused_equals_step_then_ode(G, faces):
    """gcmx_step_ode in the product default (FMA) build == gcmx_step /
    gcmx_step_faces then gcmx_ode_maxwell, bitwise (the ODE folded into the
    stores multiplies the same values the separate pass would), and within the
    tolerance of the oracle's stages + MaxwellViscosityOde (Ode.hpp:28-37)."""
    import math
    from gcm_amd.gcmx import QUANTITY_CODES as q
    fc = [[(q["Sxx"], 0.0), (q["Sxy"], 0.0), (q["Sxz"], 0.0)], None,
          [(q["Syy"], -0.3), (q["Syz"], 0.0)], [(q["Vy"], 0.1)],
          [(q["Szz"], 0.0), (q["Sxz"], 0.0), (q["Syz"], 0.0)], None] if faces else None
    b = oracle_body(3, 2, [6, 20, 32])
    random_state(b, seed=11, ghosts=False)
    a, c = fma_ctx(G, b), fma_ctx(G, b)
    f = math.exp(-0.9 / 3.0)
    for _ in range(3):
        if faces:
            a.step_faces(0.9, fc)
        else:
            a.step(0.9)
        a.ode_maxwell(0.9, [3.0])
        c.step_ode(0.9, [3.0], fc)
        if not faces:
            for s in range(3):
                b.stage(s, 0.9)
            iv = b.inner_view()
            iv[..., 3:] = iv[..., 3:] * f
    assert c.last_ode_fused and c.last_path == "fused"
    assert np.array_equal(a.download(), c.download())
    if not faces:
        check(c, b, "FMA step_ode")
    a.close(); c.close()


@pytest.mark.parametrize("kind", ["rho", "E"])
def test_fma_engine_two_layers(G, monkeypatch, kind):
    """Engine.TwoLayersDifferentRho/E (TestEngine.cpp:139-296) through the C++
    engine in the product default (FMA) build: per-node materials (the HET
    one-pass step where it applies), within the tolerance of the oracle engine."""
    from gcm_amd import _gcm_host as H
    from tests.taskspec import host_task, oracle_task, spec
    monkeypatch.setenv("GCMX_FP", "fma")
    rho0, lam0, mu0 = 1, 2, 0.8
    rho, lam, mu = (0.5, lam0, mu0) if kind == "rho" else (rho0, 0.5 * lam0, 0.5 * mu0)
    s = spec(3, 2, [1, 1, 1], {0: ([16, 12, 64], [0, 0, 0])}, 0.9, (rho0, lam0, mu0), snaps=6,
             inhomogeneities=[(("box", (-1, -1, 31.5), (100, 100, 100)), (rho, lam, mu))],
             quantities=[(("sphere", 5.0, (8, 6, 20)), "PRESSURE", 10.0)])
    he = H.Engine(host_task(s))
    he.run()
    assert he.last_path(0) == "fused"  # k_step_tx2<..., HET>
    oe = O.Engine(oracle_task(s))
    oe.run()
    assert he.steps == oe.steps_done
    got = he.pde(0)
    want = oe.bodies[0].pde.reshape(got.shape)
    r = rel_l2(got, want)
    assert r <= TOL, r
