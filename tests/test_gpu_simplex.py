"""The simplex stage on the GPU (gsx_* through gcm_amd._gcm_host.SimplexEngine) against
the oracle's restatement of the reference simplex engine, bitwise, on jittered Kuhn
meshes of the unit cube -- including Courant numbers that send inner-node feet out
through border faces (space-time interpolation, common.hpp:102-129) -- and the
reference's own engine test TestSimplexGcm.ZeroInitialization (TestSimplexGcm.cpp:29-53)."""
import numpy as np
import pytest

from tests.simplex_spec import host_task, oracle_engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    from gcm_amd import _gcm_host
    return _gcm_host


@pytest.fixture(params=[1, 8], ids=["lanes1", "lanes8"])
def lanes(request):
    """gsx_set_node_lanes: one thread per node, or eight lanes per node (the
    automatic choice below 131 072 nodes, i.e. for every mesh here)."""
    return request.param


def engine(H, t, lanes):
    e = H.SimplexEngine(t)
    e.set_node_lanes(lanes)
    return e


@pytest.mark.parametrize("n,courant,jitter,seed,steps", [(4, 1.0, 0.1, 7, 3), (4, 2.0, 0.1, 7, 2),
                                                         (6, 1.3, 0.15, 9, 2)])
def test_simplex_engine_matches_oracle(H, lanes, n, courant, jitter, seed, steps):
    t = host_task(n, courant, jitter, seed, vector=[0.1 * i for i in range(9)])
    p = H.simplex_plans(t)
    e = engine(H, t, lanes)
    assert e.time_step == p["tau"]
    o = oracle_engine(p, courant)
    e.run_steps(steps)
    for _ in range(steps):
        o.step()
    got = e.pde()
    want = np.array(o.u)
    assert np.array_equal(got, want), f"{int((got != want).sum())} values differ"
    assert np.abs(got).max() > 0


def test_simplex_zero_state_stays_zero(H):
    """TestSimplexGcm.ZeroInitialization: Engine::run from a zero state stays zero."""
    t = host_task(4, pressure=0.0)
    e = H.SimplexEngine(t)
    e.run()
    assert e.steps == 3
    assert not np.any(e.pde())


from tests.simplex_spec import FREE_BORDER, MIXED_BORDER  # noqa: E402


@pytest.mark.parametrize("border,n,courant,steps", [(FREE_BORDER, 4, 1.0, 3), (MIXED_BORDER, 4, 1.3, 3),
                                                    (FREE_BORDER, 5, 2.0, 2)],
                         ids=["free-c1", "mixed-c1.3", "free-c2"])
def test_simplex_border_correctors_match_oracle(H, lanes, border, n, courant, steps):
    """BorderCorrectorInRiemannInvariants (GLOBAL_BASIS) + the plain correction at
    the start of every step: GPU == oracle bitwise (the cube task's free surface,
    main.cpp:209-220, and a time-dependent FIXED_VELOCITY patch)."""
    t = host_task(n, courant, 0.1, 7, border=border)
    p = H.simplex_plans(t)
    e = engine(H, t, lanes)
    o = oracle_engine(p, courant, border)
    assert len(o.corrected) == len(p["border_plan"]["nodes"]) > 0
    e.run_steps(steps)
    for _ in range(steps):
        o.step()
    got, want = e.pde(), np.array(o.u)
    assert np.array_equal(got, want), f"{int((got != want).sum())} values differ"
    # the corrector changed the border values relative to no correction
    e0 = H.SimplexEngine(host_task(n, courant, 0.1, 7))
    e0.run_steps(steps)
    assert not np.array_equal(e0.pde()[p["border"]], got[p["border"]])


from tests.simplex_spec import fracture_task  # noqa: E402


@pytest.mark.parametrize("courant,steps", [(1.0, 3), (1.7, 2)])
def test_fracture_layer_matches_oracle(H, lanes, courant, steps):
    """BASELINE config 5 (meshes/layers_with_fracture.off): the layer with the
    fracture cavity, free surface on the box and on the fracture faces
    (border correctors), GPU == oracle bitwise."""
    t = fracture_task((16, 16, 8), courant)
    p = H.simplex_plans(t)
    e = engine(H, t, lanes)
    o = oracle_engine(p, courant, FREE_BORDER)
    e.run_steps(steps)
    for _ in range(steps):
        o.step()
    got, want = e.pde(), np.array(o.u)
    assert np.array_equal(got, want), f"{int((got != want).sum())} values differ"
    assert np.abs(got).max() > 0


from tests.simplex_spec import layered_task, oracle_multi  # noqa: E402


@pytest.mark.parametrize("n,courant,steps,border", [(6, 1.0, 3, None), (6, 1.7, 2, None),
                                                    (5, 1.3, 2, MIXED_BORDER)],
                         ids=["c1", "c1.7", "mixed-c1.3"])
def test_layered_adhesion_contact_matches_oracle(H, lanes, n, courant, steps, border):
    """Two bodies of different materials glued by ADHESION: the contact correctors
    (the 3 + 3 system, the 6 x 6 GSL system of a one-sided node and the averaged
    pair) between the bodies' node and inner phases, the plain contact correction
    at every step, border correctors on the outer surface: GPU == oracle bitwise."""
    t = layered_task(n, courant, border=border)
    p = H.simplex_plans(t)
    e = engine(H, t, lanes)
    assert e.number_of_bodies == 2 and e.time_step == p["tau"]
    o = oracle_multi(p, courant, border=border if border is not None else FREE_BORDER)
    e.run_steps(steps)
    for _ in range(steps):
        o.step()
    for i in range(2):
        got, want = e.pde(i), np.array(o.bodies[i].u)
        assert np.array_equal(got, want), f"body {i}: {int((got != want).sum())} values differ"
    # adhesion holds at the contact nodes: equal velocities across the contact
    c = p["contacts"][0]
    va, vb = e.pde(0)[c["nodes_a"], :3], e.pde(1)[c["nodes_b"], :3]
    assert np.abs(va).max() > 0
    assert np.abs(va - vb).max() <= 1e-12 * max(1.0, np.abs(va).max())


def test_simplex_engine_writes_vtu_snapshots(H, tmp_path, monkeypatch):
    """Engine::run with the VTK snapshotter: one .vtu per body and snapshot step
    (snapshots/vtk/mesh<id>core00snap<step>.vtu), holding the layer of that step."""
    from tests.helpers import read_vtu
    monkeypatch.chdir(tmp_path)
    t = layered_task(4, 1.0, snaps=2)
    t.add_snapshotter("VTK")
    t.set_vtk_quantities(["PRESSURE"])
    e = H.SimplexEngine(t)
    e.run()
    assert e.steps == 2
    for body in (0, 1):
        for step in (0, 1, 2):
            f = tmp_path / "snapshots" / "vtk" / f"mesh{body}core00snap{step:04d}.vtu"
            assert f.exists(), f
        arrays, pts, conn, _, _ = read_vtu(str(tmp_path / "snapshots" / "vtk" /
                                                f"mesh{body}core00snap0002.vtu"))
        assert np.array_equal(arrays["Velocity"], e.pde(body)[:, :3].astype(np.float32))


def test_inm_mesh_engine_matches_oracle(H, lanes, tmp_path):
    """INM_MESHER (InmMeshLoader.hpp): a two-material tetrahedral mesh read from an
    INM file, per-cell materials as body ids, ADHESION contact between them:
    GPU == oracle bitwise."""
    from tests.simplex_spec import write_inm
    P, C, G = H.simplex_triangulation(layered_task(5, 1.0, jitter=0.15, seed=11))
    path = tmp_path / "mesh.out"
    write_inm(path, P, C, G)
    t = layered_task(5, 1.0, inm=path)
    p = H.simplex_plans(t)
    e = engine(H, t, lanes)
    o = oracle_multi(p, 1.0)
    e.run_steps(2)
    for _ in range(2):
        o.step()
    for i in range(2):
        got, want = e.pde(i), np.array(o.bodies[i].u)
        assert np.array_equal(got, want), f"body {i}: {int((got != want).sum())} values differ"


@pytest.mark.parametrize("workload", ["cube", "layered"])
def test_graph_replayed_steps_equal_individual_calls(H, lanes, workload):
    """gsx_step (one step captured into a HIP graph per layer state and replayed)
    == the individual gsx_stage_nodes / gsx_contact_correct / gsx_stage_finish
    calls, bitwise, over enough steps to replay both layer parities, with
    time-dependent border values, and for two bodies with a contact (streams of
    both bodies in one graph)."""
    from tests.simplex_spec import MIXED_BORDER, host_task, layered_task
    import numpy as np
    mk = (lambda: host_task(6, 1.0, 0.1, 7, border=MIXED_BORDER)) if workload == "cube" else \
        (lambda: layered_task(5, 1.0))
    def run(replay):  # one engine at a time: Clock is process-global, as in the reference
        e = engine(H, mk(), lanes)
        e.set_replay_steps(replay)
        out = []
        for chunk in (1, 2, 3):
            e.run_steps(chunk)
            out.append([e.pde(body) for body in range(e.number_of_bodies)])
        return out
    a, b = run(True), run(False)
    for k, (xa, xb) in enumerate(zip(a, b)):
        for body, (pa, pb) in enumerate(zip(xa, xb)):
            assert np.array_equal(pa, pb), f"{workload} body {body} after chunk {k}"


@pytest.mark.parametrize("mode", [1, 2], ids=["border+inner", "gradient+border+inner"])
@pytest.mark.parametrize("case", ["free-c2", "mixed-c1.3", "fracture-c1.7", "plain-c1"])
def test_one_launch_stage_equals_two_launches(H, case, mode):
    """gsx_stage's one-launch stage (k_sx_stage_l8: border and inner groups side by
    side, inner feet that interpolate in space-time with border nodes' new
    invariants wait for exactly those nodes) == the border launch followed by
    the inner launch, bitwise, with space-time feet present (Courant > 1)."""
    if case == "free-c2":
        mk = lambda: host_task(5, 2.0, 0.1, 7, border=FREE_BORDER)  # noqa: E731
    elif case == "mixed-c1.3":
        mk = lambda: host_task(4, 1.3, 0.1, 7, border=MIXED_BORDER)  # noqa: E731
    elif case == "fracture-c1.7":
        mk = lambda: fracture_task((16, 16, 8), 1.7)  # noqa: E731
    else:
        mk = lambda: host_task(6, 1.0, 0.15, 9, vector=[0.1 * i for i in range(9)])  # noqa: E731
    out = []
    for fuse in (mode, 0):
        e = H.SimplexEngine(mk())
        e.set_node_lanes(8)
        e.set_stage_fusion(fuse)
        info = [e.stage_plan_info(0, s) for s in range(3)]
        e.run_steps(3)
        e.sync()
        out.append((e.pde(), e.fused_stages))
    (fused, n_fused), (split, n_split) = out
    assert n_fused == 9 and n_split == 0
    assert all(f for f, _ in info)
    if case in ("free-c2", "fracture-c1.7"):
        # the hand-off protocol is exercised: inner feet wait for border nodes' wn
        assert sum(w for _, w in info) > 0, info
    assert np.array_equal(fused, split), f"{int((fused != split).sum())} values differ"
    assert np.abs(fused).max() > 0


def test_automatic_stage_fusion_equals_fixed_mode(H):
    """the engine's default fusion mode (-1) measures modes 1
    and 2 on its first steps (an untimed warm-up step before each mode's 8
    steps between stream synchronisations) and keeps the faster; the modes give identical results, so
    a run through the choice equals a run in mode 1, bitwise.  The engine also
    counts every launch of a step (gsx_launch_count) for the launch floor."""
    mk = lambda: fracture_task((12, 12, 6), 1.0)  # noqa: E731
    steps = 1 + 2 * 8 + 3
    out = []
    for fuse in (-1, 1):
        e = H.SimplexEngine(mk())
        e.set_node_lanes(8)
        e.set_stage_fusion(fuse)
        assert e.fusion_tuning == (fuse < 0)
        l0 = e.launches
        e.run_steps(steps)
        e.sync()
        out.append((e.pde(), e.stage_fusion, e.fusion_tuning, e.fusion_times_ms, e.launches - l0))
    (auto, mode, tuning, times, launches), (fixed, mode1, _, _, launches1) = out
    assert not tuning and mode in (1, 2) and mode1 == 1
    assert times[0] > 0 and times[1] > 0
    assert (mode == 2) == (times[1] < 0.97 * times[0])
    assert launches > 0 and launches1 > 0 and launches1 % steps == 0
    assert np.array_equal(auto, fixed), f"{int((auto != fixed).sum())} values differ"
    assert np.abs(fixed).max() > 0


@pytest.mark.timeout(300)
def test_one_launch_stage_above_block_cap_completes(H):
    """k_sx_stage_l8 takes its work index from an atomic
    ticket at block start instead of blockIdx.x, so a block waits only on work
    that blocks already running took -- no assumption on the order the hardware
    dispatches workgroups in.  Mode 3 lifts the 4096-block cap: a 53^3-vertex
    cube (eight lanes per node: > 4 600 blocks of border and inner groups, with
    space-time feet waiting on border nodes at Courant 2) completes without any
    wait timing out (run_steps checks the error word) and equals the separate
    launches bitwise."""
    out = []
    for fuse in (3, 0):
        e = H.SimplexEngine(host_task(52, 2.0, 0.1, 7, border=FREE_BORDER))
        e.set_node_lanes(8)
        e.set_stage_fusion(fuse)
        info = [e.stage_plan_info(0, s) for s in range(3)]
        e.run_steps(2)
        e.sync()
        out.append((e.pde(), e.fused_stages))
    (fused, n_fused), (split, n_split) = out
    assert n_fused == 6 and n_split == 0
    assert sum(w for _, w in info) > 0, info
    assert np.array_equal(fused, split), f"{int((fused != split).sum())} values differ"


def test_one_launch_stage_timeout_is_reported(H):
    """A device wait of the one-launch stage that gives up (forced here: a wait
    budget < 0 makes every wait report a timeout) must not hand stale results to
    the host as success: run_steps (which ends with gsx_sync) and gsx_download
    raise; the error is reported once and cleared."""
    e = H.SimplexEngine(host_task(5, 2.0, 0.1, 7, border=FREE_BORDER))
    e.set_node_lanes(8)
    e.set_stage_fusion(1)
    assert sum(w for _, w in (e.stage_plan_info(0, s) for s in range(3))) > 0
    e.set_wait_budget(-1)
    with pytest.raises(Exception, match="timed out"):
        e.run_steps(1)
    e.set_wait_budget(1 << 20)
    e.run_steps(1)  # reported once, cleared, and a healthy launch reports nothing
    e.set_wait_budget(-1)
    e.run_steps(1, check=False)
    with pytest.raises(Exception, match="timed out"):
        e.pde()  # gsx_download


def _raw_simplex_plan(G, border, inner, wn_vertex):
    """A hand-made 8-node stage plan through the C-ABI: ZERO feet everywhere
    except one inner node's foot 0, a SPACETIME foot whose weights multiply the
    NEW invariants of `wn_vertex` (slot 3)."""
    import ctypes
    L = G.lib()

    class Foot(ctypes.Structure):
        _fields_ = [("kind", ctypes.c_int), ("v", ctypes.c_int * 4), ("slot", ctypes.c_int * 4),
                    ("lam", ctypes.c_double * 4), ("q", ctypes.c_double * 3)]
    N = 8
    vp = ctypes.c_void_p
    L.gsx_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(vp)]
    L.gsx_set_matrices.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    L.gsx_set_gradient_plan.argtypes = [vp] + [ctypes.c_void_p] * 6
    L.gsx_set_stage_plan.argtypes = [vp, ctypes.c_int, ctypes.POINTER(Foot), ctypes.POINTER(ctypes.c_double),
                                     ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_int)]
    L.gsx_stage.argtypes = [vp, ctypes.c_int]
    L.gsx_stage_plan_info.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    L.gsx_last_stage_fused.argtypes = [vp, ctypes.POINTER(ctypes.c_int)]
    L.gsx_set_node_lanes.argtypes = [vp, ctypes.c_int]
    L.gsx_sync.argtypes = [vp]
    L.gsx_destroy.argtypes = [vp]
    L.gsx_destroy.restype = None
    dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    coords = np.random.default_rng(1).random((N, 3))
    ctx = vp()
    G._check(L.gsx_create(0, N, dp(coords), ctypes.byref(ctx)))
    eye = np.tile(np.eye(9).reshape(-1), 3)
    G._check(L.gsx_set_matrices(ctx, dp(eye), dp(eye)))
    # gradient plan: every node one neighbour (the next), unit weight, identity normal matrix
    off = np.arange(N + 1, dtype=np.int32)
    nb = ((np.arange(N) + 1) % N).astype(np.int32)
    rows = (coords[nb] - coords).reshape(-1).copy()
    wts = np.ones(N)
    M = np.tile(np.eye(3).reshape(-1), N)
    det = np.ones(N)
    G._check(L.gsx_set_gradient_plan(ctx, off.ctypes.data, nb.ctypes.data, rows.ctypes.data, wts.ctypes.data,
                                     M.ctypes.data, det.ctypes.data))
    feet = (Foot * (N * 6))()
    for i in range(N * 6):
        feet[i].kind = 3  # GSX_FOOT_ZERO
    f = feet[inner[0] * 6 + 0]
    f.kind = 2  # GSX_FOOT_SPACETIME over the face (wn_vertex, border[0], border[0])
    f.v[0], f.v[1], f.v[2] = wn_vertex, border[0], border[0]
    f.slot[0], f.slot[1], f.slot[2], f.slot[3] = 3, 0, 0, 0
    f.lam[0], f.lam[1], f.lam[2], f.lam[3] = 0.5, 0.5, 0.0, 0.0
    shift = np.zeros(18)
    bl = np.array(border, dtype=np.int32)
    il = np.array(inner, dtype=np.int32)
    for st in range(3):
        G._check(L.gsx_set_stage_plan(ctx, st, feet, dp(shift), len(bl),
                                      bl.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), len(il),
                                      il.ctypes.data_as(ctypes.POINTER(ctypes.c_int))))
    G._check(L.gsx_set_node_lanes(ctx, 8))
    fus, waits = ctypes.c_int(), ctypes.c_int()
    G._check(L.gsx_stage_plan_info(ctx, 0, ctypes.byref(fus), ctypes.byref(waits)))
    G._check(L.gsx_stage(ctx, 0))
    G._check(L.gsx_sync(ctx))
    fused = ctypes.c_int()
    G._check(L.gsx_last_stage_fused(ctx, ctypes.byref(fused)))
    L.gsx_destroy(ctx)
    return fus.value, waits.value, fused.value


def test_unfusable_plan_runs_two_launches():
    """gsx_set_stage_plan's fusable check decides the launch shape: an inner foot
    that reads the new invariants of a node OUTSIDE the border list (nothing in
    the launch would ever publish them) makes the plan unfusable, and gsx_stage
    then runs the border and inner halves as two launches; the same foot over a
    border node is fusable, waits, and runs as one launch."""
    import gcm_amd.gcmx as G
    border, inner = [0, 1], [2, 3, 4, 5, 6, 7]
    assert _raw_simplex_plan(G, border, inner, wn_vertex=5) == (0, 1, 0)
    assert _raw_simplex_plan(G, border, inner, wn_vertex=1) == (1, 1, 1)


from tests.simplex_spec import CUBE_BORDER, cube_task  # noqa: E402


@pytest.mark.timeout(600)
def test_cube_task_matches_oracle_across_the_load_switch(H):
    """BASELINE config 4 (parseTaskCube, launcher/main.cpp:547-639): meshes/cube.off
    at spatial step 0.05 (9 261 vertices), Courant 1, free surface everywhere and
    the traction (0, 0, t < 0.25 ? -1 : 0) on the x <= 0.01 face.  10 steps of
    tau = 0.0336 run past t = 0.25, where the load switches off; the GPU (the
    default engine: eight lanes, one launch per stage) equals the oracle bitwise
    at the switch step and at the end."""
    t = cube_task()
    p = H.simplex_plans(t)
    e = H.SimplexEngine(t)
    o = oracle_engine(p, 1.0, CUBE_BORDER)
    tau = e.time_step
    assert tau == p["tau"]
    switch = next(k for k in range(1, 20) if k * tau >= 0.25)  # b(t + tau) turns 0 at this step
    done = 0
    for target in (switch + 1, 10):
        e.run_steps(target - done)
        for _ in range(target - done):
            o.step()
        done = target
        got, want = e.pde(), np.array(o.u)
        assert np.array_equal(got, want), f"step {done}: {int((got != want).sum())} values differ"
    assert e.fused_stages > 0
    assert np.abs(got).max() > 0


def test_device_interpolation_known_answers():
    """The simplex kernels' device interpolation (csrc/simplex.hip tet_hybrid /
    tet_linear, what k_sx_inner / k_sx_border run per foot) on the reference's
    own known-answer inputs (TestInterpolator.cpp:183-282), with the weights the
    host plans compute: bitwise equal to the oracle's hybridInterpolate and
    linear form; exact for a linear f (TetrahedronInterpolator.linear, within
    EQUALITY_TOLERANCE * |f(q)|) and for a quadratic f wherever the hybrid limiter
    kept the quadratic value (TetrahedronInterpolator.quadratic); interpolateInOwner's
    answer 1 (:247-257) and the quadraticMinMax input's hybrid value 1.5 (:274-282)."""
    from gcm_amd import _gcm_host as H
    from gcm_amd import gcmx as G
    from oracle import simplex as S
    from tests.test_simplex_cpu import _f3, _g3, _q3, tet_known_answer_cases
    cases = tet_known_answer_cases(1000, seed=183)
    C = np.array([c for c, _ in cases], dtype=np.float64)
    Q = np.array([q for _, q in cases], dtype=np.float64)
    lam = np.array([H.tet_barycentric(*[list(x) for x in c], list(q)) for c, q in cases])
    for fn, gr, name in ((_f3, lambda x: (5.0, 8.0, -4.0), "linear"), (_q3, _g3, "quadratic")):
        V = np.array([[fn(x) for x in c] for c, _ in cases], dtype=np.float64)
        Gr = np.array([[gr(x) for x in c] for c, _ in cases], dtype=np.float64)
        hyb, lin = G.test_interpolate(V, Gr, C, Q, lam)
        want_h = [S.tet_hybrid_lam(tuple(l), c, list(v), [tuple(g) for g in gg], q)
                  for l, (c, q), v, gg in zip(lam, cases, V, Gr)]
        want_l = [S.tet_linear_lam(tuple(l), list(v)) for l, v in zip(lam, V)]
        assert np.array_equal(hyb, np.array(want_h)), name
        assert np.array_equal(lin, np.array(want_l)), name
        exact = np.array([fn(q) for _, q in cases])
        tol = S.EQUALITY_TOLERANCE * np.abs(exact)
        if name == "linear":
            assert np.all(np.abs(lin - exact) <= tol) and np.all(np.abs(hyb - exact) <= tol)
        else:
            quad = np.array([S.tet_quadratic_lam(tuple(l), c, list(v), [tuple(g) for g in gg], q)
                             for l, (c, q), v, gg in zip(lam, cases, V, Gr)])
            kept = hyb == quad
            assert kept.sum() > 100
            assert np.all(np.abs(hyb[kept] - exact[kept]) <= tol[kept])
    # interpolateInOwner (space-time foot): owner weights from the host pick, value 1
    c6 = [[0, 0, 0], [0, 1, 0], [1, 0, 0], [0, 0, 1], [0, 1, 1], [1, 0, 1]]
    v6 = [1.0, 1.0, 1.0, 1.0, 1e100, 1e100]
    slots, lw = H.tet_owner_pick([list(map(float, p)) for p in c6], [0.1, 0.1, 0.1])
    v4 = np.array([[v6[s] for s in slots]])
    _, lin = G.test_interpolate(v4, np.zeros((1, 4, 3)), np.zeros((1, 4, 3)), np.zeros((1, 3)), np.array([lw]))
    assert lin[0] == 1.0
    # quadraticMinMax's input through the hybrid form: the limiter fires, linear value 1.5
    c = [(0, 0, 1), (0, 1, 0), (1, 0, 0), (-1, -1, -1)]
    lq = H.tet_barycentric(*[list(map(float, x)) for x in c], [0.0, 0.0, 0.0])
    hyb, _ = G.test_interpolate(np.array([[1.0, 1, 1, 3]]), np.array([[(0, 0, 2), (0, 2, 0), (2, 0, 0), (-2, -2, -2)]],
                                dtype=np.float64), np.array([c], dtype=np.float64), np.zeros((1, 3)), np.array([lq]))
    assert hyb[0] == 1.5 == S.tet_hybrid(c, [1, 1, 1, 3], [(0, 0, 2), (0, 2, 0), (2, 0, 0), (-2, -2, -2)], (0, 0, 0))
