"""The C++ host mirror (Task -> createEngine -> cubic::Engine<D>::run) on the GPU,
restating the reference's engine tests (src/test/sequence/TestEngine.cpp) and
checking every run bitwise against the oracle engine on the same Task."""
import math

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import seq_sum
from tests.taskspec import host_task, oracle_task, spec

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    from gcm_amd import _gcm_host
    return _gcm_host


@pytest.fixture(scope="module")
def G():
    import gcm_amd.gcmx as G
    return G


def inner(arr, bs, D):
    sl = tuple(slice(bs, -bs) for _ in range(D))
    return arr[sl]


def run_both(H, s, steps=None):
    oe = O.Engine(oracle_task(s))
    he = H.Engine(host_task(s))
    if steps is None:
        oe.run(); he.run()
        assert he.steps == oe.steps_done
    else:
        oe.run(max_steps=steps); he.run_steps(steps)
    return oe, he


def assert_bodies_equal(oe, he, s, inner_only=False):
    """Bitwise equal bodies; inner_only: the inner nodes only -- the one-pass step
    forms y/z face ghosts in registers and never writes them, while the oracle's
    ghost layers keep the last per-stage fill (scratch no output reads)."""
    for b in oe.bodies:
        got = he.pde(b.id)
        want = b.pde.reshape(got.shape)
        if inner_only:
            got, want = inner(got, s["bs"], s["D"]), inner(want, s["bs"], s["D"])
        assert np.array_equal(got, want), f"body {b.id}: {int((got != want).sum())} values differ"


def sphere_spec(N=32, snaps=5):
    return spec(3, 2, [1, 1, 1], {0: ([N] * 3, [0] * 3)}, 0.9, (4, 2, 1), snaps=snaps,
                quantities=[(("sphere", N / 4, (N / 2,) * 3), "PRESSURE", 10.0)])


def test_engine_anchor_3d(H):
    """SURVEY.md §8c anchor through Task -> Engine::run (fused path)."""
    s = sphere_spec()
    he = H.Engine(host_task(s))
    assert he.path(0) == "fused"
    he.run()
    assert he.steps == 5
    got = he.pde(0)
    total = seq_sum(inner(got, 2, 3))
    assert total == -63401.220461788325


def test_engine_anchor_1d(H):
    s = spec(1, 2, [1], {0: ([10000], [0])}, 0.9, (4, 2, 1), snaps=1000,
             waves=[(("box", (1000, -1, -1), (2000, 1, 1)), "P_FORWARD", 0, "Vx", 1.0)])
    he = H.Engine(host_task(s))
    he.run_steps(1000)
    v = inner(he.pde(0), 2, 1)
    tot = 0.0
    tot2 = 0.0
    for x in v.reshape(-1).tolist():
        tot += x
        tot2 += x * x
    assert tot == -2997.0000000000014 and tot2 == 16914.932549439342
    he2 = H.Engine(host_task(s))
    he2.run()
    assert he2.steps == 1001  # Clock semantics (AbstractEngine.cpp:35-43)


def adhesion(two):
    X, Y = 21, 41
    cubics = {0: ([X, Y], [0, 0]), 1: ([X, Y], [0, Y])} if two else {0: ([X, 2 * Y], [0, 0])}
    return spec(2, 2, [1, 0.25], cubics, 0.9, (4, 2, 0.5), snaps=70,
                waves=[(("box", (-1000, 2.5, -1000), (1000, 7.5, 1000)), "P_FORWARD", 1,
                        "PRESSURE", 1.0)])


def test_engine_adhesion_contact(H):
    """Engine.AdhesionContact (TestEngine.cpp:27-87): bitwise split == unsplit, and == oracle."""
    two = H.Engine(host_task(adhesion(True)))
    two.run()
    one = H.Engine(host_task(adhesion(False)))
    one.run()
    a0, a1, aa = inner(two.pde(0), 2, 2), inner(two.pde(1), 2, 2), inner(one.pde(0), 2, 2)
    assert np.array_equal(aa[:, :41], a0) and np.array_equal(aa[:, 41:], a1)
    oe = O.Engine(oracle_task(adhesion(True)))
    oe.run()
    assert_bodies_equal(oe, two, adhesion(True))


def xcontact(two):
    """Two 3-D bodies stacked along x (a contact along the stage-0 axis) or one."""
    X, Y, Z = 12, 20, 64
    cubics = {0: ([X, Y, Z], [0, 0, 0]), 1: ([X, Y, Z], [X, 0, 0])} if two else {0: ([2 * X, Y, Z], [0, 0, 0])}
    return spec(3, 2, [1, 1, 1], cubics, 0.9, (4, 2, 1), snaps=6,
                quantities=[(("sphere", 6.0, (X - 1.5, Y / 2, Z / 2)), "PRESSURE", 10.0)])


@pytest.mark.parametrize("stacks", [True, False])
def test_engine_contact_along_x_one_pass(H, monkeypatch, stacks):
    """3-D bodies whose contacts all lie along x.  By default the chain runs as
    one grid (a stack, like y / z chains: inner nodes bitwise, the ghost layers
    at the contact are scratch).  With GCMX_NO_STACKS=1 the engine copies every
    contact's ghost planes first (they read the neighbours' E_n,
    Engine.cpp:99-107) and then runs one gcmx_step per body -- the one-pass
    kernel, since an x-ghost copy keeps it admissible -- and equals the oracle
    with ghosts included.  Two bodies == one body and == the oracle, bitwise."""
    if not stacks:
        monkeypatch.setenv("GCMX_NO_STACKS", "1")
    two = H.Engine(host_task(xcontact(True)))
    two.run()
    assert two.last_path(0) == "fused" and two.last_path(1) == "fused"
    one = H.Engine(host_task(xcontact(False)))
    one.run()
    a0, a1, aa = inner(two.pde(0), 2, 3), inner(two.pde(1), 2, 3), inner(one.pde(0), 2, 3)
    assert np.any(aa != 0)
    assert np.array_equal(aa[:12], a0) and np.array_equal(aa[12:], a1)
    oe = O.Engine(oracle_task(xcontact(True)))
    oe.run()
    assert oe.steps_done == two.steps
    assert_bodies_equal(oe, two, xcontact(True), inner_only=stacks)


def test_engine_run_statement(H):
    """Engine.runStatement (TestEngine.cpp:91-136): bs 5, Courant 4.5, exact translation."""
    s = spec(2, 5, [7.0 / 19, 3.0 / 39], {0: ([20, 40], [0, 0])}, 4.5, (4, 2, 0.5), snaps=9,
             required_time=100.0,
             waves=[(("box", (-1, 0.1125, -1), (8, 0.6375, 1)), "S1_FORWARD", 1, "Vx", 1.0)])
    he = H.Engine(host_task(s))
    expected = inner(he.pde(0), 5, 2)[10, 3].copy()
    he.run()
    actual = inner(he.pde(0), 5, 2)[10, 22]
    for a, b in zip(expected, actual):
        assert 4 * (a - b) ** 2 / ((a + b) ** 2 + 1e-9) < 1e-18
    oe, he2 = run_both(H, s)
    assert_bodies_equal(oe, he2, s)


@pytest.mark.parametrize("kind", ["rho", "E"])
def test_engine_two_layers(H, kind):
    """Engine.TwoLayersDifferentRho/E (TestEngine.cpp:139-296) on the GPU (per-node
    materials: generic kernel), reflection within 1e-2 and bitwise == oracle."""
    rho0, lam0, mu0 = 1, 2, 0.8
    for i in range(5):
        if kind == "rho":
            rho, lam, mu = 0.25 * 2 ** i * rho0, lam0, mu0
        else:
            rho, lam, mu = rho0, 0.25 * 2 ** i * lam0, 0.25 * 2 ** i * mu0
        s = spec(2, 3, [2.0 / 49, 1.0 / 99], {0: ([50, 100], [0, 0])}, 1.5, (rho0, lam0, mu0),
                 inhomogeneities=[(("box", (-10, 0.5 - 1e-5, -10), (10, 10, 10)), (rho, lam, mu))],
                 snaps=0, required_time=0.24,
                 waves=[(("box", (-1, 0.015, -1), (4, 0.455, 1)), "P_FORWARD", 1, "Vy", -2.0)])
        he = H.Engine(host_task(s))
        assert he.path(0) == "generic"
        init = inner(he.pde(0), 3, 2)[25, 25].copy()
        he.run()
        refl = inner(he.pde(0), 3, 2)[25, 25]
        E0 = mu0 * (3 * lam0 + 2 * mu0) / (lam0 + mu0); Z0 = math.sqrt(E0 * rho0)
        E = mu * (3 * lam + 2 * mu) / (lam + mu); Z = math.sqrt(E * rho)
        assert abs(refl[4] / init[4] - (Z - Z0) / (Z + Z0)) < 1e-2
        assert abs(refl[1] / init[1] - (Z0 - Z) / (Z + Z0)) < 1e-2
        oe = O.Engine(oracle_task(s))
        oe.run()
        assert_bodies_equal(oe, he, s)


def test_engine_border_conditions_time_dependent(H):
    """Cubic border conditions with time dependencies, overlapping conditions and
    PRESSURE (BorderConditions.hpp:46-114), 2-D and 3-D: bitwise == oracle."""
    f = lambda t: 0.5 * math.sin(3 * t)
    s2 = spec(2, 2, [0.5, 0.25], {0: ([30, 25], [0, 0])}, 0.8, (4, 2, 1), snaps=12,
              waves=[(("box", (3, -1, -1), (8, 100, 1)), "P_FORWARD", 0, "PRESSURE", 1.0)],
              borders={0: [(0, ("infinite",), {"Sxx": f, "Sxy": lambda t: 0.0}),
                           (1, ("box", (-1, -1, -1), (7.2, 100, 1)), {"PRESSURE": lambda t: 0.1 * t}),
                           (1, ("box", (4.1, -1, -1), (100, 100, 1)), {"Vy": lambda t: -0.2})]})
    oe, he = run_both(H, s2)
    assert_bodies_equal(oe, he, s2)
    s3 = spec(3, 2, [1, 1, 1], {0: ([10, 9, 12], [0, 0, 0])}, 0.9, (4, 2, 1), snaps=6,
              quantities=[(("sphere", 3, (5, 4, 6)), "PRESSURE", 2.0)],
              borders={0: [(2, ("infinite",), {"Szz": lambda t: 0.0, "Sxz": lambda t: 0.0,
                                               "Syz": lambda t: 0.0}),
                           (0, ("cylinder", 3, (0, 4, 6), (20, 4, 6)), {"Vx": f})]})
    oe, he = run_both(H, s3)
    assert he.path(0) == "fused"  # the cylinder covers part of face x-: a face map
    assert_bodies_equal(oe, he, s3, inner_only=True)


def test_engine_setup_areas_waves_vectors_3d(H):
    """MaterialsCondition / InitialCondition with every area kind, vectors,
    waves and quantities summed in order, three materials: bitwise == oracle."""
    s = spec(3, 2, [0.5, 1.0, 0.75], {0: ([14, 11, 16], [2, 0, 1])}, 0.7, (4, 2, 1),
             inhomogeneities=[(("sphere", 2.5, (4, 5, 6)), (2, 1, 1.5)),
                              (("cylinder", 1.5, (0, 0, 0), (8, 11, 12)), (3, 0.5, 2))],
             snaps=4,
             vectors=[(("box", (1, 1, 1), (6, 8, 9)), [0.1 * i for i in range(9)])],
             waves=[(("box", (2, 2, 2), (5, 6, 8)), "S2_BACKWARD", 2, "Vy", 0.7),
                    (("sphere", 3, (3, 5, 7)), "P_FORWARD", 1, "PRESSURE", -1.0)],
             quantities=[(("infinite",), "Syz", 0.3)])
    oe, he = run_both(H, s)
    assert_bodies_equal(oe, he, s)


def test_engine_bad_courant_raises(H):
    s = spec(3, 2, [1, 1, 1], {0: ([6, 6, 6], [0, 0, 0])}, 2.5, (4, 2, 1), snaps=1)
    he = H.Engine(host_task(s))
    with pytest.raises(H.GcmException):
        he.run()


@pytest.mark.parametrize("D,tau0_b,path", [(3, None, "fused"), (2, 7.0, "generic"), (1, None, "generic"),
                                           (3, 0.0, "generic")])
def test_engine_maxwell_ode(H, D, tau0_b, path):
    """Task bodies with MAXWELL_VISCOSITY (Engine.cpp:28-31, 115-119; Ode.hpp:24-38):
    Task -> Engine::run on the GPU == the oracle engine, bitwise."""
    from tests.test_oracle import _maxwell_spec
    s = _maxwell_spec(D, 3.0, tau0_b)
    he = H.Engine(host_task(s))
    assert he.path(0) == path
    oe, he = run_both(H, s)
    assert_bodies_equal(oe, he, s)
    # one material on the one-pass path: the ODE rides in the step's store epilogue
    assert he.ode_fused(0) == (path == "fused")


@pytest.mark.parametrize("faces", [False, True])
def test_step_ode_fused_equals_step_then_ode(G, faces):
    """gcmx_step_ode == gcmx_step / gcmx_step_faces followed by gcmx_ode_maxwell,
    bitwise, with the ODE folded into k_step_tx2's stores (one material; tau0 = 0
    gives the factor exp(-inf) = 0).  Several materials keep the separate pass
    (test_engine_maxwell_ode: the generic path)."""
    from tests.helpers import context_for, oracle_body, random_state
    q = G.QUANTITY_CODES
    fc = [[(q["Sxx"], 0.0), (q["Sxy"], 0.0), (q["Sxz"], 0.0)], None,
          [(q["Syy"], -0.3), (q["Syz"], 0.0)], [(q["Vy"], 0.1)],
          [(q["Szz"], 0.0), (q["Sxz"], 0.0), (q["Syz"], 0.0)], None] if faces else None
    for tau0, fused, sizes in ((3.0, True, [6, 20, 32]), (0.0, True, [6, 20, 32]), (3.0, True, [5, 12, 1024])):
        b = oracle_body(3, 2, sizes)  # Z = 1024: the z split's epilogue (k_step_tx2 and k_zseam)
        random_state(b, seed=11, ghosts=False)
        a, c = context_for(b), context_for(b)
        for _ in range(3):
            if faces:
                a.step_faces(0.9, fc)
            else:
                a.step(0.9)
            a.ode_maxwell(0.9, [tau0])
            c.step_ode(0.9, [tau0], fc)
        assert c.last_ode_fused == fused and c.last_path == "fused"
        assert np.array_equal(a.download(), c.download())
        a.close(); c.close()


def test_engine_rejects_uncompilable_odes(H):
    """Only MaxwellViscosityOde compiles in the reference (Ode.hpp:50, 75)."""
    s = spec(2, 2, [1, 1], {0: ([8, 8], [0, 0])}, 0.9, (4, 2, 1), snaps=1,
             odes={0: ["CONTINUAL_DAMAGE"]})
    with pytest.raises(Exception):
        H.Engine(host_task(s))


def test_engine_snapshotters(H, tmp_path, monkeypatch):
    """AbstractEngine::run with VTK and SLICESNAP snapshotters (AbstractEngine.cpp:30-46,
    Snapshotter.hpp:46-77, VtkSnapshotter.hpp:26-77, SliceSnapshotter.hpp:37-90):
    file set, .vts contents, z-axis slice and detector series == the oracle's states."""
    from tests.helpers import read_vts
    from tests.test_snapshot_cpu import _expected
    monkeypatch.chdir(tmp_path)
    N = 12
    s = spec(3, 2, [1, 1, 1], {0: ([N] * 3, [0] * 3)}, 0.9, (4, 2, 1), snaps=3, steps_per_snap=2,
             quantities=[(("sphere", 3.0, (6.0, 6.0, 6.0)), "PRESSURE", 10.0)])
    t = host_task(s)
    t.add_snapshotter("VTK")
    t.add_snapshotter("SLICESNAP")
    t.set_vtk_quantities(["PRESSURE"])
    t.set_detector(["Szz"], ("box", (-1, -1, -1), (7.5, 100, 100)), 0)
    t.output_directory = "out"
    he = H.Engine(t)
    he.run()
    assert he.steps == 6
    oe = O.Engine(oracle_task(s))
    times, seismo, time = [], [], 0.0
    for step in range(7):
        if step:
            oe.run(max_steps=step)
            time += oe.time_step
        if step % 2:
            continue
        b = oe.bodies[0]
        stem = f"snapshots/out/%s/mesh0core00snap{step:04d}"
        dims, arrays, points = read_vts(stem % "vtk" + ".vts")
        vel, pts, q, _ = _expected(b, [("PRESSURE", "pressure")])
        assert np.array_equal(arrays["Velocity"], vel) and np.array_equal(points, pts)
        assert np.array_equal(arrays["pressure"][:, 0], q["pressure"])
        inn = b.inner_view()
        col = inn[N // 2, N // 2, :, 2]
        want = "".join(f"{float(z):g}\t{float(v):g}\t\n" for z, v in zip(range(N), col))
        assert open(stem % "zaxis" + ".txt").read() == want
        face = inn[:, :, N - 1, 8]  # Szz on the top face, x < 7.5
        vals = [float(face[x, y]) for x in range(N) for y in range(N) if x < 7.5]
        acc = 0.0
        for v in vals:
            acc += v
        times.append(time)
        seismo.append(float(np.float32(acc / len(vals))))
        want = "".join(f"{a:g}\t{c:g}\t\n" for a, c in zip(times, seismo))
        assert open(stem % "detector" + ".txt").read() == want


def ystack(bodies_sizes, axis=1, materials=None, maxwell=False, at=None):
    """3-D bodies stacked along `axis` (adhesion contacts over whole faces), a
    pressure sphere centred at `at` along it (default: 1.5 before the first contact)."""
    X, Y, Z = 10, 12, 64
    cubics, off = {}, 0
    for i, w in enumerate(bodies_sizes):
        sz, st = [X, Y, Z], [0, 0, 0]
        sz[axis], st[axis] = w, off
        cubics[i] = (sz, st)
        off += w
    c = [X / 2, Y / 2, Z / 2]
    c[axis] = bodies_sizes[0] - 1.5 if at is None else at
    return spec(3, 2, [1, 1, 1], cubics, 0.9, (4, 2, 1), snaps=5,
                inhomogeneities=materials or [],
                quantities=[(("sphere", 5.0, tuple(c)), "PRESSURE", 10.0)],
                odes={i: ["MAXWELL_VISCOSITY"] for i in cubics} if maxwell else None)


@pytest.mark.parametrize("axis,widths", [(0, [6, 6]), (0, [5, 4, 7]), (1, [6, 6]), (1, [5, 4, 7]), (2, [32, 32]),
                                         (2, [20, 24, 20])])
def test_engine_stack_equals_one_body(H, monkeypatch, axis, widths):
    """VERDICT r3 missing 4: contacts along y / z.  Bodies stacked along y or z
    with adhesion contacts over whole faces run as ONE grid (a stack): every
    ContactCopier copy fills exactly the ghost layers the stack's own stage reads
    (Engine.cpp:99-107), so the inner nodes equal one body (TestEngine.cpp:27-87's
    split == unsplit) and the oracle's copy-then-stage engine, bitwise, and the
    step runs the one-pass kernel.  GCMX_NO_STACKS=1 (separate bodies, per-stage
    copies) gives the same inner nodes."""
    s = ystack(widths, axis)
    he = H.Engine(host_task(s))
    he.run()
    assert all(he.last_path(i) == "fused" for i in range(len(widths)))
    oe = O.Engine(oracle_task(s))
    oe.run()
    assert he.steps == oe.steps_done
    for b in oe.bodies:
        got = inner(he.pde(b.id), 2, 3)
        want = inner(b.pde.reshape(he.pde(b.id).shape), 2, 3)
        assert np.array_equal(got, want), f"body {b.id}: {int((got != want).sum())} differ"
    one = H.Engine(host_task(ystack([sum(widths)], axis, at=widths[0] - 1.5)))
    one.run()
    whole = inner(one.pde(0), 2, 3)
    parts = np.concatenate([inner(he.pde(i), 2, 3) for i in range(len(widths))], axis=axis)
    assert np.array_equal(parts, whole)
    monkeypatch.setenv("GCMX_NO_STACKS", "1")
    sep = H.Engine(host_task(s))
    sep.run()
    assert sep.last_path(0) == ("fused" if axis == 0 else "split")  # x contacts: per-body one pass
    for i in range(len(widths)):
        assert np.array_equal(inner(sep.pde(i), 2, 3), inner(he.pde(i), 2, 3))


def test_engine_stack_two_materials_and_maxwell(H):
    """A stack whose bodies carry different materials (per-node materials: the
    HET one-pass step) and the Maxwell ODE, against the oracle engine bitwise."""
    mats = [(("box", (-1, 6.5, -1), (100, 100, 100)), (2.0, 1.0, 0.5, 30.0))]
    s = ystack([7, 5], 1, materials=mats, maxwell=True)
    s["material"] = (4, 2, 1, 50.0)
    he = H.Engine(host_task(s))
    he.run()
    oe = O.Engine(oracle_task(s))
    oe.run()
    for b in oe.bodies:
        got = inner(he.pde(b.id), 2, 3)
        want = inner(b.pde.reshape(he.pde(b.id).shape), 2, 3)
        assert np.array_equal(got, want), f"body {b.id}: {int((got != want).sum())} differ"
