"""Pins the CPU oracle to the reference.

Every test here restates a known-answer test of the reference
(src/test/sequence/*.cpp) or checks a bitwise sanity anchor that the survey
measured by running the reference itself.
CPU only.
"""
import math

import numpy as np
import pytest

from oracle import oracle as O


def approx_equal(f1, f2, tol=1e-9):
    """Utils::approximatelyEqual (util/Utils.hpp:35-42)."""
    rel2 = 4 * (f1 - f2) * (f1 - f2) / ((f1 + f2) * (f1 + f2) + tol)
    return rel2 < tol * tol


def seq_sums(a):
    s = 0.0
    s2 = 0.0
    for x in np.asarray(a).reshape(-1).tolist():
        s += x
        s2 += x * x
    return s, s2


# ------------------------------------------------------- survey anchors ----

def test_anchor_3d_pressure_sphere_bitwise():
    """3-D N=32, (4,2,1), bs=2, tau=0.9, pressure sphere p=10,
    r=N/4 at N/2, 5 steps: sum and sum of squares are bitwise the reference's."""
    N = 32
    t = O.Task(D=3, border_size=2, h=[1, 1, 1], cubics={0: ([N] * 3, [0] * 3)}, courant=0.9,
               default_material=O.Material(4, 2, 1), number_of_snaps=5,
               ic_quantities=[(("sphere", N / 4, (N / 2,) * 3), "PRESSURE", 10.0)])
    e = O.Engine(t)
    assert e.time_step == 0.9
    assert e.run() == 5
    s, s2 = seq_sums(e.bodies[0].inner_view())
    assert s == -63401.220461788325
    assert s2 == 225405.1366274695


def test_anchor_1d_p_wave_bitwise():
    """1-D N=10000, P_FORWARD wave Vx=1 on x in (1000,2000), 1000 steps."""
    t = O.Task(D=1, border_size=2, h=[1], cubics={0: ([10000], [0])}, courant=0.9,
               default_material=O.Material(4, 2, 1), number_of_snaps=1000,
               ic_waves=[(("box", (1000, -1, -1), (2000, 1, 1)), "P_FORWARD", 0, "Vx", 1.0)])
    e = O.Engine(t)
    e.run(max_steps=1000)
    s, s2 = seq_sums(e.bodies[0].inner_view())
    assert s == -2997.0000000000014
    assert s2 == 16914.932549439342


def test_step_count_clock_semantics():
    """AbstractEngine::run counts steps by `time += tau` vs tau*N (AbstractEngine.cpp:20-43):
    for tau = 0.9 and N = 1000 the reference runs 1001 steps."""
    assert O.step_count(0.9, 0.9 * 1000 * 1) == 1001
    assert O.step_count(0.9, 0.9 * 5 * 1) == 5


# --------------------------------------------------------- matrices --------

def test_survey_printed_matrices_axis0():
    """U / U1 of (4,2,1) along axis 0 (probe print of the reference)."""
    U, U1, L = O.isotropic_elastic_matrices(3, 4, 2, 1)
    expU = {0: {0: 1, 3: -.25}, 1: {0: 1, 3: .25}, 2: {1: -1, 4: .5}, 3: {1: -1, 4: -.5},
            4: {2: -1, 5: .5}, 5: {2: -1, 5: -.5}, 6: {7: 1}, 7: {6: 1, 8: -1},
            8: {3: -1, 6: 1, 8: 1}}
    expU1 = {0: {0: .5, 1: .5}, 1: {2: -.5, 3: -.5}, 2: {4: -.5, 5: -.5}, 3: {0: -2, 1: 2},
             4: {2: 1, 3: -1}, 5: {4: 1, 5: -1}, 6: {0: -1, 1: 1, 7: .5, 8: .5}, 7: {6: 1},
             8: {0: -1, 1: 1, 7: -.5, 8: .5}}
    for exp, M in ((expU, U[0]), (expU1, U1[0])):
        for r in range(9):
            for c in range(9):
                assert M[r, c] == exp[r].get(c, 0.0), (r, c)
    assert list(L[0]) == [1, -1, .5, -.5, .5, -.5, 0, 0, 0]
    assert int(np.count_nonzero(U)) == 3 * 18 and int(np.count_nonzero(U1)) == 3 * 21


def _A_matrix(D, rho, lam, mu, s):
    """ElasticModel::constructGcmMatrix's A (ElasticModel.hpp:374-397), l = 1, n = e_s."""
    M = O.pde_size(D)
    n = np.zeros(D); n[s] = 1
    A = np.zeros((M, M))
    sig = lambda i, j: D + O._sym_index(D, i, j)
    for i in range(D):
        vec = np.zeros(M)
        for j in range(D):
            vec[sig(i, j)] = -1 * n[j] / rho
        A[i, :] = vec
    for i in range(D):
        vec = np.zeros(M)
        for j in range(D):
            vec[sig(i, j)] = -1 * mu * n[j]
        for j in range(D):
            vec[sig(j, j)] += -1 * (lam + (i == j) * mu) * n[i]
        A[:, i] = vec
    return A


@pytest.mark.parametrize("D", [1, 2, 3])
def test_isotropic_decomposition(D):
    """IsotropicGcmMatrix (TestGcmMatrices.cpp:64-106) / checkDecomposition
    (util/math/GridCharacteristicMethod.hpp:60-69): A U1 = U1 L, U A = L U, U U1 = I."""
    rng = np.random.default_rng(7)
    for _ in range(200):
        rho = rng.uniform(0.01, 100); lam = rng.uniform(1, 1e6); mu = rng.uniform(1, 1e6)
        U, U1, L = O.isotropic_elastic_matrices(D, rho, lam, mu)
        for s in range(D):
            A = _A_matrix(D, rho, lam, mu, s)
            Lm = np.diag(L[s])
            eps = 1e-9 * 100 * 1000
            for X, Y in ((A @ U1[s], U1[s] @ Lm), (U[s] @ A, Lm @ U[s]),
                         (U[s] @ U1[s], np.eye(O.pde_size(D)))):
                for a, b in zip(X.reshape(-1), Y.reshape(-1)):
                    assert approx_equal(a, b, eps)
            assert approx_equal(np.trace(A), L[s].sum(), 1e-7)


def test_max_eigenvalue_cubic_grid_initialize():
    """CubicGrid.initialize (TestCubicGrid.cpp:12-37): max eigenvalue of (4,2,0.5) 2-D."""
    t = O.Task(D=2, border_size=3, h=[1, 1], cubics={0: ([7, 9], [0, 0])}, courant=1,
               default_material=O.Material(4, 2, 0.5), number_of_snaps=1)
    b = O.Engine(t).bodies[0]
    assert abs(b.maximal_eigenvalue - 0.866025404) < 1e-9
    assert np.all(b.inner_view() == 0.0)


def test_diagonal_multiply_exact():
    """Linal.diagonalMultiply (TestLinal.cpp:869-890): == (A*B)(k,k) exactly."""
    rng = np.random.default_rng(3)
    for _ in range(50):
        A = rng.uniform(-1, 1, (9, 9)); B = rng.uniform(-1, 1, (9, 9))
        r = O.diagonal_multiply(A, B)
        for k in range(9):
            acc = A[k, 0] * B[0, k]
            for n in range(1, 9):
                acc += A[k, n] * B[n, k]
            assert r[k] == acc


# ----------------------------------------------------- interpolation -------

def _q_range(stop, step):
    q = 0.0
    while q <= stop:
        yield q
        q += step


def test_interpolator_const():
    N = 5
    for i in range(21):
        for q in _q_range(float(i), 0.2):
            src = np.array([[math.sinh(j - N / 2) for j in range(N)]] * (i + 1))
            res = O.interpolate(src, q)
            for j in range(N):
                assert abs(res[j] - math.sinh(j - N / 2)) < 1e-9


def test_interpolator_linear():
    N = 9
    for k in range(21):
        for q in _q_range(float(k), 0.2):
            src = np.array([[(j - N / 2) * i + 2 * (j - N / 2) for j in range(N)]
                            for i in range(k + 1)], dtype=float)
            res = O.interpolate(src, q)
            for j in range(N):
                assert abs(res[j] - ((j - N / 2) * q + 2 * (j - N / 2))) < 1e-9


def test_interpolator_quadratic():
    for q in _q_range(2.0, 0.1):
        src = np.zeros((3, 9))
        src[:, 0] = [0, 1, 4]; src[:, 1] = [0, -1, -4]; src[:, 2] = [-3, 15, 89]
        res = O.interpolate(src, q)
        assert abs(res[0] - q * q) < 1e-9
        assert abs(res[1] + q * q) < 1e-9
        assert abs(res[2] - (7 * (2 * q) ** 2 - 5 * (2 * q) - 3)) < 1e-9


def test_interpolator_minmax_exact_clamp():
    src = np.array([[-9.0, 9.0], [-1.0, 1.0], [-1.0, 1.0]])
    res = O.min_max_interpolate(src, 1.5)
    assert res[0] == -1.0 and res[1] == 1.0


def test_interpolator_minmax_fifth_order():
    for q in _q_range(5.0, 0.1):
        src = np.zeros((6, 2)); src[3:, 0] = 1
        if int(q) >= 5:  # the reference reads src[6] here (undefined behaviour)
            continue
        res = O.min_max_interpolate(src, q)
        if q <= 2:
            assert abs(res[0]) < 1e-9
        elif q < 3:
            assert 0 < res[0] < 1
        else:
            assert abs(res[0] - 1) < 1e-9


def test_interpolator_tenth_order():
    f = lambda x: x ** 10 + 4 * x ** 9 - 25 * x ** 7 + 2 * x ** 5 - 3 * x * x + 5
    q = 0.0
    while q < 11.0:
        src = np.array([[f(i), 0.0] for i in range(11)])
        res = O.interpolate(src, q)
        assert abs(res[0] - f(q)) <= abs(res[0]) * 1e-9 * 1e3
        q += 0.1


def test_interpolator_exceptions():
    with pytest.raises(ValueError):
        O.min_max_interpolate(np.zeros((2, 5)), -0.3)
    with pytest.raises(ValueError):
        O.min_max_interpolate(np.zeros((2, 5)), 2.5)


def test_interpolate_values_around():
    """GridCharacteristicMethodCubicGrid.interpolateValuesAround
    (TestGridCharacteristicMethod.cpp:15-70): 3x3 2-D grid, bs=1, pressure -1
    at node (1,1); columns for dx = (-1, 1, -0.5, 0.5, 0).  The two |dx| = 1
    columns make the reference read past its 2-point vector inside the limiter
    (UB), so they are checked through the Newton part alone."""
    t = O.Task(D=2, border_size=1, h=[1, 1], cubics={0: ([3, 3], [0, 0])}, courant=1,
               default_material=O.Material(2, 2, 1), number_of_snaps=1,
               ic_quantities=[(("sphere", 0.1, (1, 1, 0)), "PRESSURE", -1.0)])
    b = O.Engine(t).bodies[0]
    v = b.inner_view()
    for x in range(3):
        for y in range(3):
            c = 1.0 if (x, y) == (1, 1) else 0.0
            assert list(v[x, y]) == [0.0, 0.0, c, 0.0, c]
    dx = [-1, 1, -0.5, 0.5, 0]
    for stage in (0, 1):
        m = np.zeros((5, 5))
        for k, d in enumerate(dx):
            shift = 1 if d > 0 else -1
            src = []
            for i in range(2):
                it = [1, 1]; it[stage] += shift * i
                src.append(b.pde[b.flat_index(np.array(it))])
            src = np.array(src)
            q = abs(d) / 1.0
            m[:, k] = O.interpolate(src, q) if q >= 1 else O.min_max_interpolate(src, q)
        for i in range(5):
            assert m[i, 0] == 0.0 and m[i, 1] == 0.0
            assert m[0, i] == 0.0 and m[1, i] == 0.0 and m[3, i] == 0.0
        assert m[2, 2] == 0.5 and m[2, 3] == 0.5 and m[4, 2] == 0.5 and m[4, 3] == 0.5
        assert m[2, 4] == 1.0 and m[4, 4] == 1.0


# ------------------------------------------------------------ engine -------

def adhesion_task(two_bodies: bool):
    X, Y = 21, 41
    cubics = {0: ([X, Y], [0, 0]), 1: ([X, Y], [0, Y])} if two_bodies else {0: ([X, 2 * Y], [0, 0])}
    return O.Task(D=2, border_size=2, h=[1, 0.25], cubics=cubics, courant=0.9,
                  default_material=O.Material(4, 2, 0.5), number_of_snaps=70,
                  ic_waves=[(("box", (-1000, 2.5, -1000), (1000, 7.5, 1000)), "P_FORWARD", 1,
                             "PRESSURE", 1.0)])


def test_engine_adhesion_contact_bitwise():
    """Engine.AdhesionContact (TestEngine.cpp:27-87): two stacked bodies with an
    adhesion contact == one body, bitwise (coordinates and PDE values)."""
    two = O.Engine(adhesion_task(True)); two.run()
    one = O.Engine(adhesion_task(False)); one.run()
    first, second = two.bodies
    allb = one.bodies[0]
    va, v0, v1 = allb.inner_view(), first.inner_view(), second.inner_view()
    Y = 41
    assert np.array_equal(va[:, :Y], v0)
    assert np.array_equal(va[:, Y:], v1)
    it = allb.inner_indices()
    assert np.any(va != 0)


def run_statement_task():
    return O.Task(D=2, border_size=5, h=[7.0 / 19, 3.0 / 39], cubics={0: ([20, 40], [0, 0])},
                  courant=4.5, default_material=O.Material(4, 2, 0.5), number_of_snaps=9,
                  required_time=100.0,
                  ic_waves=[(("box", (-1, 0.1125, -1), (8, 0.6375, 1)), "S1_FORWARD", 1, "Vx",
                             1.0)])


def test_engine_run_statement():
    """Engine.runStatement (TestEngine.cpp:91-136): Courant 4.5 with bs 5 moves an
    S-wave 19 nodes exactly: pde{10,3} at t0 ~= pde{10,22} at the end."""
    e = O.Engine(run_statement_task())
    b = e.bodies[0]
    expected = b.inner_view()[10, 3].copy()
    assert np.any(expected != 0)
    e.run()
    actual = b.inner_view()[10, 22]
    for a, x in zip(expected, actual):
        assert approx_equal(a, x)


def two_layers_task(rho, lam, mu):
    rho0, lam0, mu0 = 1, 2, 0.8
    return O.Task(D=2, border_size=3, h=[2.0 / 49, 1.0 / 99], cubics={0: ([50, 100], [0, 0])},
                  courant=1.5, default_material=O.Material(rho0, lam0, mu0),
                  inhomogeneities=[(("box", (-10, 0.5 - 1e-5, -10), (10, 10, 10)),
                                    O.Material(rho, lam, mu))],
                  number_of_snaps=0, required_time=0.24,
                  ic_waves=[(("box", (-1, 0.015, -1), (4, 0.455, 1)), "P_FORWARD", 1, "Vy", -2.0)])


@pytest.mark.parametrize("kind", ["rho", "E"])
def test_engine_two_layers_reflection(kind):
    """Engine.TwoLayersDifferentRho / DifferentE (TestEngine.cpp:139-296): the reflected
    wave matches the impedance ratio within 1e-2 (per-node material switch)."""
    rho0, lam0, mu0 = 1, 2, 0.8
    for i in range(5):
        if kind == "rho":
            rho, lam, mu = 0.25 * 2 ** i * rho0, lam0, mu0
        else:
            rho, lam, mu = rho0, 0.25 * 2 ** i * lam0, 0.25 * 2 ** i * mu0
        e = O.Engine(two_layers_task(rho, lam, mu))
        b = e.bodies[0]
        init = b.inner_view()[25, 25].copy()
        assert np.any(init != 0)
        e.run()
        refl = b.inner_view()[25, 25]
        E0 = mu0 * (3 * lam0 + 2 * mu0) / (lam0 + mu0); Z0 = math.sqrt(E0 * rho0)
        E = mu * (3 * lam + 2 * mu) / (lam + mu); Z = math.sqrt(E * rho)
        syy = 2 + O._sym_index(2, 1, 1)
        assert abs(refl[syy] / init[syy] - (Z - Z0) / (Z + Z0)) < 1e-2
        assert abs(refl[1] / init[1] - (Z0 - Z) / (Z + Z0)) < 1e-2


def test_border_condition_pressure_clears_vector():
    """BorderConditions::handleBorderPoint with PRESSURE (BorderConditions.hpp:94-114,
    VelocitySigmaVariables.hpp:106-111): the ghost is the mirrored inner vector,
    then PRESSURE's setter clears it and writes -(-p_inner + 2 f) on the diagonal."""
    t = O.Task(D=2, border_size=2, h=[1, 1], cubics={0: ([6, 5], [0, 0])}, courant=0.5,
               default_material=O.Material(4, 2, 1), number_of_snaps=1,
               border_conditions={0: [O.BorderCondition(0, ("infinite",),
                                                        {"PRESSURE": lambda t: 0.25})]})
    e = O.Engine(t)
    b = e.bodies[0]
    rng = np.random.default_rng(0)
    b.pde[:] = rng.uniform(-1, 1, b.pde.shape)
    b.apply_border(0, 0.0)
    for y in range(5):
        for a in (1, 2):
            inner = b.pde[b.flat_index(np.array([a, y]))]
            ghost = b.pde[b.flat_index(np.array([-a, y]))]
            p_in = (-(0.0 + inner[2] + inner[4])) / 2
            gv = -p_in + 2 * 0.25
            assert list(ghost) == [0.0, 0.0, -gv, 0.0, -gv]


def test_random_field_is_splitmix():
    v = O.splitmix_uniform(0x5EED, 0)
    assert -1.0 <= v < 1.0
    assert O.splitmix_uniform(0x5EED, 0) == v
    assert O.splitmix_uniform(0x5EED, 1) != v


# ------------------------------------------------------------ Maxwell ODE --
# MaxwellViscosityOde (rheology/ode/Ode.hpp:24-38), applied by cubic::Engine after
# the stages of every step (engine/cubic/Engine.cpp:115-119).  The reference has
# no test of its own for it: parity unpinned beyond the defining identity below.

def _maxwell_spec(D, tau0_a, tau0_b=None):
    from tests.taskspec import spec
    N = [12] * D
    inh = []
    if tau0_b is not None:
        inh = [(("box", (-1, -1, -1), (5.5, 100, 100)), (4, 2, 1, tau0_b))]
    return spec(D, 2, [1.0] * D, {0: (N, [0] * D)}, 0.9, (4, 2, 1, tau0_a), inhomogeneities=inh,
                snaps=3, quantities=[(("sphere", 3.0, (6.0,) * 3), "PRESSURE", 2.0)],
                vectors=[(("box", (2, 2, 2), (9, 9, 9)), [0.5] * O.pde_size(D))],
                odes={0: ["MAXWELL_VISCOSITY"]})


@pytest.mark.parametrize("D,tau0_b", [(1, None), (2, 7.0), (3, None), (3, 0.0)])
def test_maxwell_ode_scales_stress_after_each_step(D, tau0_b):
    """One step with the ODE == the same step without it, then every stress component
    of every inner node times exp(-tau / tau0[material]) (tau0 = 0 gives 0)."""
    from tests.taskspec import oracle_task
    s = _maxwell_spec(D, 3.0, tau0_b)
    with_ode = O.Engine(oracle_task(s))
    s2 = dict(s); s2["odes"] = {}
    plain = O.Engine(oracle_task(s2))
    for _ in range(2):
        with_ode.run(max_steps=with_ode.steps_done + 1)
        plain.run(max_steps=plain.steps_done + 1)
        b, p = with_ode.bodies[0], plain.bodies[0]
        tau = with_ode.time_step
        flat = b.flat_index(b.inner_indices())
        for node in flat[:: max(1, len(flat) // 97)]:
            t0 = b.tau0[b.mat_id[node]]
            f = math.exp(-tau / t0) if t0 != 0 else 0.0
            assert np.array_equal(b.pde[node, :D], p.pde[node, :D])
            assert np.array_equal(b.pde[node, D:], p.pde[node, D:] * f)
        p.pde[:] = b.pde  # continue both from the same state
