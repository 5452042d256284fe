"""GPU parity: libgcmx.so (through its C-ABI) against the oracle, bitwise.

Bit-exact is the bar (integer-exact arithmetic order, no FMA contraction): the
comparison is IEEE equality, which identifies +0 and -0 (the skipped exact-zero
matrix terms can only change the sign of an exact zero).
"""
import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import (assert_same, context_for, oracle_body, random_materials, random_state,
                           seq_sum)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G():
    import gcm_amd
    gcm_amd.lib()
    return gcm_amd


CASES = [
    (1, 1, [37]), (1, 2, [300]), (1, 3, [65]),
    (2, 1, [9, 13]), (2, 2, [21, 70]), (2, 3, [17, 5]), (2, 5, [20, 40]),
    (3, 1, [7, 9, 11]), (3, 2, [12, 10, 70]), (3, 3, [6, 8, 19]),
]


@pytest.mark.parametrize("D,bs,sizes", CASES)
def test_generic_stages_random_with_ghosts(G, D, bs, sizes):
    """Every stage of two time steps, random state including ghost layers."""
    b = oracle_body(D, bs, sizes, h=[1.0, 0.5, 2.0][:D])
    random_state(b, seed=D * 10 + bs, ghosts=True)
    ctx = context_for(b, path=G.PATH_GENERIC)
    tau = 0.9 * 0.5 / 1.0  # Courant 0.9 on the smallest h
    for step in range(2):
        for s in range(D):
            b.stage(s, tau)
            ctx.stage(s, tau)
            assert_same(ctx, b, f"D={D} bs={bs} step {step} stage {s}")


@pytest.mark.parametrize("bs,sizes", [(1, [5, 6, 7]), (2, [13, 17, 70]), (2, [9, 4, 300]),
                                      (3, [10, 11, 64]), (2, [140, 3, 5])])
def test_split_stages_3d(G, bs, sizes):
    b = oracle_body(3, bs, sizes)
    random_state(b, seed=bs + sizes[2], ghosts=True)
    ctx = context_for(b, path=G.PATH_SPLIT)
    assert ctx.effective_path == "split"
    for step in range(2):
        for s in range(3):
            b.stage(s, 0.9)
            ctx.stage(s, 0.9)
            assert_same(ctx, b, f"split bs={bs} sizes={sizes} step {step} stage {s}")


@pytest.mark.parametrize("bs,sizes", [(2, [12, 10, 70]), (2, [9, 150, 300]), (1, [4, 3, 64]),
                                      (3, [130, 7, 100]), (2, [5, 66, 520]), (3, [3, 5, 512]),
                                      (3, [3, 4, 1024])])
def test_fused_step_3d(G, bs, sizes):
    """gcmx_step on the fused path (X march + fused Y/Z) == three oracle stages."""
    b = oracle_body(3, bs, sizes)
    random_state(b, seed=sum(sizes), ghosts=False)
    ctx = context_for(b, path=G.PATH_AUTO)
    assert ctx.effective_path == "fused"
    for step in range(3):
        for s in range(3):
            b.stage(s, 0.9)
        ctx.step(0.9)
        assert_same(ctx, b, f"fused bs={bs} sizes={sizes} step {step}")


@pytest.mark.parametrize("bs,sizes", [(2, [5, 9, 1024]), (1, [4, 6, 1024]), (2, [3, 130, 1024])])
def test_zsplit_step_matches_oracle(G, bs, sizes):
    """Rows longer than 512: the z-split one-pass step -- two
    512-lane parts per row, the Z stage of the nodes next to the cut from the
    parts' Y results (k_zseam) -- == three oracle stages, bitwise, odd X included."""
    b = oracle_body(3, bs, sizes)
    random_state(b, seed=sum(sizes) + bs, ghosts=False)
    ctx = context_for(b, path=G.PATH_AUTO)
    ctx.profile(True)
    for step in range(3):
        for s in range(3):
            b.stage(s, 0.9)
        ctx.step(0.9)
        assert_same(ctx, b, f"z split bs={bs} sizes={sizes} step {step}")
    k = ctx.profile_read()["fused_xyz"]["kernel"]
    assert k.startswith("k_step_tx2<") and "ZS" in k, k
    ctx.close()


def test_zsplit_not_taken_above_courant_one(G):
    """floor(q) > 0 (Courant 1.5) keeps rows of 1024 on the one-plane k_fused_xyz,
    which still equals the oracle."""
    b = oracle_body(3, 2, [4, 6, 1024])
    random_state(b, seed=11, ghosts=False)
    ctx = context_for(b, path=G.PATH_AUTO)
    ctx.profile(True)
    for s in range(3):
        b.stage(s, 1.5)
    ctx.step(1.5)
    assert_same(ctx, b, "Courant 1.5, Z = 1024")
    assert ctx.profile_read()["fused_xyz"]["kernel"].startswith("k_fused_xyz<")
    ctx.close()


def test_fused_disabled_by_nonzero_ghosts(G):
    b = oracle_body(3, 2, [6, 6, 6])
    random_state(b, seed=1, ghosts=True)
    ctx = context_for(b)
    assert ctx.effective_path == "split"
    for s in range(3):
        b.stage(s, 0.9)
    ctx.step(0.9)
    assert_same(ctx, b, "auto path with ghosts")


@pytest.mark.parametrize("D,bs,sizes", [(2, 2, [23, 31]), (3, 2, [9, 10, 11]), (3, 3, [7, 6, 40])])
def test_heterogeneous_materials(G, D, bs, sizes):
    mats = ((4.0, 2.0, 1.0), (1.0, 2.0, 0.8), (2.5, 0.0, 3.0))
    b = oracle_body(D, bs, sizes, materials=mats, courant=0.9)
    random_materials(b, seed=5)
    random_state(b, seed=6, ghosts=True)
    ctx = context_for(b)
    assert ctx.effective_path == "generic"
    tau = 0.9 / np.sqrt((3.0 + 6.0) / 2.5)  # Courant 0.9 on the fastest material
    for step in range(2):
        for s in range(D):
            b.stage(s, tau)
            ctx.stage(s, tau)
            assert_same(ctx, b, f"hetero D={D} step {step} stage {s}")


@pytest.mark.parametrize("path", ["generic", "split", "fused"])
def test_large_courant_multi_cell(G, path):
    """Courant 2.5 with borderSize 3: feet two cells away (k = floor(q) = 2)."""
    p = {"generic": G.PATH_GENERIC, "split": G.PATH_SPLIT, "fused": G.PATH_FUSED}[path]
    b = oracle_body(3, 3, [8, 9, 70])
    random_state(b, seed=11, ghosts=False)
    ctx = context_for(b, path=p)
    tau = 2.5
    for step in range(2):
        for s in range(3):
            b.stage(s, tau)
        if path == "fused":
            ctx.step(tau)
        else:
            for s in range(3):
                ctx.stage(s, tau)
        assert_same(ctx, b, f"{path} courant 2.5 step {step}")


def test_cfl_violation_is_an_error(G):
    b = oracle_body(3, 2, [6, 6, 6])
    ctx = context_for(b)
    with pytest.raises(G.GcmxError) as e:
        ctx.stage(0, 2.0)  # q = 2 = borderSize: the reference asserts / reads out of range
    assert e.value.status == 2
    with pytest.raises(ValueError):
        b.stage(0, 2.0)


def test_anchor_pressure_sphere_on_gpu(G):
    """SURVEY.md §8c anchor reproduced on the GPU through gcmx_step (fused) and
    gcmx_stage (generic): bitwise the reference's sums."""
    N = 32
    t = O.Task(D=3, border_size=2, h=[1, 1, 1], cubics={0: ([N] * 3, [0] * 3)}, courant=0.9,
               default_material=O.Material(4, 2, 1), number_of_snaps=5,
               ic_quantities=[(("sphere", N / 4, (N / 2,) * 3), "PRESSURE", 10.0)])
    for path in (G.PATH_AUTO, G.PATH_GENERIC):
        b = O.Engine(t).bodies[0]
        ctx = context_for(b, path=path)
        for _ in range(5):
            ctx.step(0.9)
        got = ctx.download()
        s = seq_sum(b.inner_view(got))
        assert s == -63401.220461788325, (path, s)


def test_fill_random_matches_oracle(G):
    b = oracle_body(3, 2, [5, 7, 9], start=[3, 0, 0])
    b.pde[:] = 0
    O.fill_random(b, [20, 7, 9], 0x5EED)
    ctx = context_for(oracle_body(3, 2, [5, 7, 9], start=[3, 0, 0]))
    ctx.fill_random([20, 7, 9], 0x5EED)
    assert_same(ctx, b, "fill_random")


def test_border_fill_matches_oracle(G):
    """cubic BorderConditions (BorderConditions.hpp:81-114) on the device."""
    D, bs = 2, 2
    t = O.Task(D=D, border_size=bs, h=[1, 1], cubics={0: ([8, 7], [0, 0])}, courant=0.9,
               default_material=O.Material(4, 2, 1), number_of_snaps=1,
               border_conditions={0: [
                   O.BorderCondition(0, ("box", (-1, 1.5, -1), (100, 4.5, 1)),
                                     {"Sxx": lambda t: 0.5, "Sxy": lambda t: -0.25}),
                   O.BorderCondition(1, ("infinite",), {"PRESSURE": lambda t: 0.125}),
               ]})
    b = O.Engine(t).bodies[0]
    random_state(b, seed=3, ghosts=True)
    ctx = context_for(b)
    qcode = {"Vx": 2, "Vy": 3, "Vz": 4, "Sxx": 5, "Sxy": 6, "Sxz": 7, "Syy": 8, "Syz": 9,
             "Szz": 10, "PRESSURE": 12}
    for direction in (0, 1):
        b.apply_border(direction, 0.0)
        for d, left, right, vals in b.border:
            if d != direction:
                continue
            qs = [qcode[q] for q, _ in vals]
            vs = [f(0.0) for _, f in vals]
            ctx.border_fill(d, -1, left, qs, vs)
            ctx.border_fill(d, +1, right, qs, vs)
        assert_same(ctx, b, f"border fill direction {direction}")


def test_adhesion_contact_two_contexts_bitwise(G):
    """Engine.AdhesionContact (TestEngine.cpp:27-87) on the device: two bodies
    joined by contact copies == one body, bitwise, and == the oracle."""
    from tests.test_oracle import adhesion_task
    two = O.Engine(adhesion_task(True))
    one = O.Engine(adhesion_task(False))
    tau = two.time_step
    nsteps = O.step_count(tau, two.required_time)
    b0, b1 = two.bodies
    c0, c1 = context_for(b0), context_for(b1)
    call = context_for(one.bodies[0])
    Y, bs = 41, 2
    for _ in range(nsteps):
        for s in range(2):
            if s == 1:  # contact direction: body0's top ghosts <- body1 rows 0..1, and back
                c0.copy_box([0, Y], [21, Y + bs], c1, [0, 0])
                c1.copy_box([0, -bs], [21, 0], c0, [0, Y - bs])
            c0.stage(s, tau); c1.stage(s, tau); call.stage(s, tau)
    two.run(); one.run()
    g0, g1, ga = c0.download(), c1.download(), call.download()
    i0, i1, ia = b0.inner_view(g0), b1.inner_view(g1), one.bodies[0].inner_view(ga)
    assert np.array_equal(ia[:, :Y], i0) and np.array_equal(ia[:, Y:], i1)
    assert np.array_equal(ia, one.bodies[0].inner_view())


@pytest.mark.parametrize("sched", ["single", "xslab", "bfirst"])
def test_x_slabs_with_copy_halo_equal_single(G, sched):
    """Slab decomposition along X (the multi-GPU layout) on one device: two
    slabs whose X ghosts are refreshed from the neighbour before every step
    (gcmx_halo_exchange_group) == one context, bitwise, on the fused path, with
    the one-launch and the three-stream X-slab step schedules."""
    N, bs, seed = 40, 2, 0x5EED
    import gcm_amd
    from gcm_amd.host import isotropic_elastic_matrices
    U, U1, L = isotropic_elastic_matrices(3, 4, 2, 1)
    full = gcm_amd.Context(3, bs, [N, N, N])
    full.set_materials(U[None], U1[None], L[None]); full.fill_random([N, N, N], seed)
    halves = []
    for r, (x0, X) in enumerate(((0, 17), (17, N - 17))):
        c = gcm_amd.Context(3, bs, [X, N, N], start=[x0, 0, 0])
        c.set_materials(U[None], U1[None], L[None]); c.fill_random([N, N, N], seed)
        c.set_schedule({"xslab": G.SCHED_XSLAB, "bfirst": G.SCHED_BFIRST}.get(sched, G.SCHED_SINGLE))
        halves.append(c)
    a, b = halves
    from gcm_amd.gcmx import halo_exchange_group
    for _ in range(3):
        halo_exchange_group([a, b])
        full.step(0.9); a.step(0.9); b.step(0.9)
    assert a.effective_path == "fused" and b.effective_path == "fused"
    fa, ga, gb = full.download(), a.download(), b.download()
    sh = lambda c, arr: arr.reshape(tuple(s + 2 * bs for s in c.sizes) + (9,))[bs:-bs, bs:-bs, bs:-bs]
    F = sh(full, fa)
    assert np.array_equal(F[:17], sh(a, ga)) and np.array_equal(F[17:], sh(b, gb))


def _slab_contexts(G, X, Y, Z, nslabs, seed, sched, rows=0):
    import gcm_amd
    from gcm_amd.host import isotropic_elastic_matrices
    U, U1, L = isotropic_elastic_matrices(3, 4, 2, 1)
    out = []
    for r in range(nslabs):
        c = gcm_amd.Context(3, 2, [X, Y, Z], start=[r * X, 0, 0])
        c.set_materials(U[None], U1[None], L[None])
        c.fill_random([X * nslabs, Y, Z], seed)
        c.set_schedule(sched, rows)
        out.append(c)
    return out


@pytest.mark.timeout(600)
def test_xslab_schedule_64x512x512_slabs_match_oracle(G):
    """BASELINE config 3's slab shape (512^3 over 8 GPUs = 64 x 512 x 512 per
    GPU) on one device: two in-process X slabs under the three-stream X-slab
    schedule (interior planes on the low-priority stream with the adaptive
    16-row chunk, both 16-row boundary sides on their own streams), halos
    refreshed by gcmx_halo_exchange_group before each step, == the oracle run
    on the undivided 128 x 512 x 512 box, bitwise (TestMPI.cpp:92-155 idea,
    ASSERT_EQ at :150)."""
    import os
    from gcm_amd.gcmx import halo_exchange_group
    X, Y, Z, bs, seed, nsteps = 64, 512, 512, 2, 0x5EED, 2
    slabs = _slab_contexts(G, X, Y, Z, 2, seed, G.SCHED_XSLAB)
    for _ in range(nsteps):
        halo_exchange_group(slabs)
        for c in slabs:
            c.step(0.9)
    assert all(c.effective_path == "fused" for c in slabs)
    got = [c.download().reshape(X + 2 * bs, Y + 2 * bs, Z + 2 * bs, 9)[bs:-bs, bs:-bs, bs:-bs]
           for c in slabs]
    for c in slabs:
        c.close()
    b = oracle_body(3, bs, [2 * X, Y, Z])
    O.fill_random(b, [2 * X, Y, Z], seed)
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    for _ in range(nsteps):
        for s in range(3):
            b.stage(s, 0.9, threads)
    want = b.inner_view()
    for r in range(2):
        assert np.array_equal(got[r], want[r * X:(r + 1) * X]), f"slab {r}"


@pytest.mark.parametrize("rows", [1, 7, 16, 128, 1000])
def test_fused_rows_per_block_any_value(G, rows):
    """The fused kernel's y chunk (gcmx_set_step_schedule rows_per_block) does
    not change results: prologue recompute of 2*BS X rows per chunk, partial
    last chunk, chunk > Y."""
    b = oracle_body(3, 2, [6, 40, 64])
    random_state(b, seed=rows, ghosts=False)
    ctx = context_for(b, path=G.PATH_AUTO)
    ctx.set_schedule(G.SCHED_SINGLE, rows)
    for step in range(2):
        for s in range(3):
            b.stage(s, 0.9)
        ctx.step(0.9)
        assert_same(ctx, b, f"rows {rows} step {step}")


@pytest.mark.parametrize("sizes", [[6, 24, 512], [5, 20, 256], [4, 12, 1024], [7, 9, 128]])
def test_fused_uni_instance_matches_oracle(G, sizes):
    """The benched specialisation k_fused_xyz<BS=2, ZT=Z, KF0, UNI> (Z == ZT,
    isotropic (4,2,1) with h = 1 on every axis: one IsoAxis for all three
    stages); [6, 24, 512] is the 512^3 bench instance (ZT = 512), three steps
    against the oracle, bitwise."""
    b = oracle_body(3, 2, sizes)
    random_state(b, seed=sum(sizes), ghosts=False)
    ctx = context_for(b, path=G.PATH_AUTO)
    assert ctx.effective_path == "fused"
    for step in range(3):
        for s in range(3):
            b.stage(s, 0.9)
        ctx.step(0.9)
        assert_same(ctx, b, f"uni sizes={sizes} step {step}")


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_full_size_256_paths_agree_and_match_oracle(G):
    """256^3 (BASELINE config 2): one step on the fused path == split == oracle."""
    import gcm_amd
    from gcm_amd.host import isotropic_elastic_matrices
    N, seed = 256, 0x5EED
    U, U1, L = isotropic_elastic_matrices(3, 4, 2, 1)
    outs = {}
    for path in (G.PATH_FUSED, G.PATH_SPLIT):
        c = gcm_amd.Context(3, 2, [N, N, N])
        c.set_materials(U[None], U1[None], L[None]); c.set_path(path)
        c.fill_random([N, N, N], seed)
        c.step(0.9)
        outs[path] = c.download()
        c.close()
    assert np.array_equal(outs[G.PATH_FUSED], outs[G.PATH_SPLIT])
    b = oracle_body(3, 2, [N, N, N])
    O.fill_random(b, [N, N, N], seed)
    for s in range(3):
        b.stage(s, 0.9, 16)
    assert np.array_equal(b.inner_view(outs[G.PATH_FUSED]), b.inner_view())


@pytest.mark.parametrize("het", [False, True])
def test_two_generation_rows_match_oracle(G, het):
    """A launch of exactly two resident blocks per CU ([256, 64, 256]: 128 plane
    pairs x 4 chunks of 16 rows = 512 blocks on 256 CUs) takes the two-generation
    row split (old blocks 20 rows, young 12; kernels_xyz.hip tx2_gen2), uniform
    and per-node media: 2 steps == the oracle, bitwise.  (On a device with another
    CU count the launch keeps equal chunks; the comparison holds either way.)"""
    sizes = [256, 64, 256]
    mats = ((4.0, 2.0, 1.0), (1.0, 2.0, 0.8)) if het else None
    b = oracle_body(3, 2, sizes, materials=mats, courant=0.9) if het else oracle_body(3, 2, sizes)
    if het:
        its = b.inner_indices()
        b.mat_id[b.flat_index(its)] = np.where(its[:, 0] < sizes[0] // 2, 0, 1).astype(np.uint8)
    random_state(b, seed=11, ghosts=False)
    ctx = context_for(b)
    assert ctx.effective_path == "fused"
    tau = 0.9 / np.sqrt((3.0 + 6.0) / 2.5) if het else 0.9
    ctx.profile(True)
    for step in range(2):
        for s in range(3):
            b.stage(s, tau, 16)
        ctx.step(tau)
        assert_same(ctx, b, f"gen2 het={het} step {step}")
    assert "k_step_tx2<2, 256" in ctx.profile_read()["fused_xyz"]["kernel"]
    ctx.close()


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_full_size_512_step_matches_oracle(G):
    """512^3 (the headline bench configuration): one step on the default path
    (k_fused_xyz<2, 512, KF0, UNI>) == the oracle at all host threads, bitwise."""
    import os
    import gcm_amd
    from gcm_amd.host import isotropic_elastic_matrices
    N, seed = 512, 0x5EED
    U, U1, L = isotropic_elastic_matrices(3, 4, 2, 1)
    c = gcm_amd.Context(3, 2, [N, N, N])
    c.set_materials(U[None], U1[None], L[None])
    c.fill_random([N, N, N], seed)
    assert c.effective_path == "fused"
    c.step(0.9)
    got = c.download()
    c.close()
    b = oracle_body(3, 2, [N, N, N])
    O.fill_random(b, [N, N, N], seed)
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    for s in range(3):
        b.stage(s, 0.9, threads)
    assert np.array_equal(b.inner_view(got), b.inner_view())


@pytest.mark.parametrize("bs,sizes,layout", [(2, [6, 20, 64], "random"), (2, [7, 9, 128], "random"),
                                             (1, [5, 12, 64], "random"), (2, [8, 16, 256], "layers"),
                                             (2, [6, 24, 512], "layers")])
def test_heterogeneous_one_pass_step_matches_oracle(G, bs, sizes, layout):
    """Per-node materials on the one-pass step (k_step_tx2<..., HET>): every node's
    three stages use its own material's tables (GridCharacteristicMethod::stage
    takes each node's matrices), applied per wave through the materials present;
    random ids put two materials in almost every lane pair (the X stage without
    shared differences), layers (x < X/2 vs x >= X/2, the TestEngine two-layer
    layout) keep waves uniform.  3 steps == the oracle's stages, bitwise."""
    mats = ((4.0, 2.0, 1.0), (1.0, 2.0, 0.8), (2.5, 0.0, 3.0))
    b = oracle_body(3, bs, sizes, materials=mats, courant=0.9)
    if layout == "random":
        random_materials(b, seed=5)
    else:
        its = b.inner_indices()
        b.mat_id[b.flat_index(its)] = np.where(its[:, 0] < sizes[0] // 2, 0, 1).astype(np.uint8)
    random_state(b, seed=6, ghosts=False)
    ctx = context_for(b)
    assert ctx.effective_path == "fused"
    tau = 0.9 / np.sqrt((3.0 + 6.0) / 2.5)  # Courant 0.9 on the fastest material: floor(q) = 0
    ctx.profile(True)
    for step in range(3):
        for s in range(3):
            b.stage(s, tau)
        ctx.step(tau)
        assert ctx.last_path == "fused"
        assert_same(ctx, b, f"HET {layout} step {step}")
    k = ctx.profile_read()
    assert "HET" in k["fused_xyz"]["kernel"], k
    ctx.close()


@pytest.mark.parametrize("faces", [False, True])
def test_heterogeneous_step_ode_fused_equals_step_then_ode(G, faces):
    """MaxwellViscosityOde (Ode.hpp:28-37) folded into the heterogeneous one-pass
    step's stores: each node's stresses times ITS material's exp(-tau / tau0[m]).
    gcmx_step_ode == gcmx_step (gcmx_step_faces) followed by gcmx_ode_maxwell's
    per-node pass, bitwise, with random ids (two materials in most lane pairs)."""
    from gcm_amd.gcmx import QUANTITY_CODES as q
    fc = [[(q["Sxx"], 0.0), (q["Sxy"], 0.0), (q["Sxz"], 0.0)], None,
          [(q["Syy"], -0.3), (q["Syz"], 0.0)], [(q["Vy"], 0.1)],
          [(q["Szz"], 0.0), (q["Sxz"], 0.0), (q["Syz"], 0.0)], None] if faces else None
    mats = ((4.0, 2.0, 1.0), (1.0, 2.0, 0.8), (2.5, 0.0, 3.0))
    b = oracle_body(3, 2, [8, 16, 64], materials=mats, courant=0.9)
    random_materials(b, seed=5)
    random_state(b, seed=6, ghosts=False)
    tau = 0.9 / np.sqrt((3.0 + 6.0) / 2.5)
    tau0 = [3.0, 0.5, 7.0]
    a, c = context_for(b), context_for(b)
    for _ in range(3):
        if faces:
            a.step_faces(tau, fc)
        else:
            a.step(tau)
        a.ode_maxwell(tau, tau0)
        c.step_ode(tau, tau0, fc)
        assert c.last_ode_fused and c.last_path == "fused"
    assert not a.last_ode_fused
    assert np.array_equal(a.download(), c.download())
    a.close(); c.close()

def test_heterogeneous_many_materials_take_per_stage_path(G):
    """More materials than the one-pass step keeps in LDS (kHetMaxMaterials = 32):
    the per-stage path with per-node matrices, still bitwise == the oracle."""
    mats = tuple((4.0 + 0.1 * i, 2.0, 1.0) for i in range(40))
    b = oracle_body(3, 2, [6, 12, 64], materials=mats, courant=0.9)
    random_materials(b, seed=9)
    random_state(b, seed=10, ghosts=False)
    ctx = context_for(b)
    for step in range(2):
        for s in range(3):
            b.stage(s, 0.9)
        ctx.step(0.9)
        assert ctx.last_path != "fused"
        assert_same(ctx, b, f"40 materials step {step}")
    ctx.close()
