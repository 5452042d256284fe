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
        e.run_steps(3)
        e.sync()
        out.append((e.pde(), e.fused_stages))
    (fused, n_fused), (split, n_split) = out
    assert n_fused == 9 and n_split == 0
    assert np.array_equal(fused, split), f"{int((fused != split).sum())} values differ"
    assert np.abs(fused).max() > 0
