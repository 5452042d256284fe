"""BASELINE config 3 on one device: X slabs of one grid as the ranks of an
in-process group (gcmx_comm_init_local), so the exchange code that RCCL drives
on a multi-GPU node -- the X-slab step schedule (interior beside the boundary
planes, the new boundary planes posted while the interior runs, the next step's
boundary kernels waiting for them) and the per-stage exchange of the split path
-- runs unchanged, with device copies in place of ncclSend/Recv.

The reference's own check of its (dead) MPI slab design is slab == sequential,
bitwise (src/test/TestMPI.cpp:92-155, ASSERT_EQ at :150; the exchange itself at
:33-50); these tests compare the slabs with one undivided context or with the
oracle, bitwise."""
import os
import threading

import numpy as np
import pytest

from oracle import oracle as O
from tests.helpers import oracle_body

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G():
    import gcm_amd.gcmx as G
    try:
        G.lib()
    except Exception as e:  # pragma: no cover
        pytest.fail(f"libgcmx.so not loadable: {e}")
    return G


def _mats():
    from gcm_amd.host import isotropic_elastic_matrices
    return isotropic_elastic_matrices(3, 4, 2, 1)


def _group(G, xs, Y, Z, seed, sched=None, path=None, bs=2):
    """Contexts for X slabs of widths `xs` of an (sum(xs), Y, Z) grid, one group."""
    import gcm_amd
    U, U1, L = _mats()
    Xg = sum(xs)
    out, x0 = [], 0
    for X in xs:
        c = gcm_amd.Context(3, bs, [X, Y, Z], start=[x0, 0, 0])
        c.set_materials(U[None], U1[None], L[None])
        c.fill_random([Xg, Y, Z], seed)
        if sched is not None:
            c.set_schedule(sched)
        if path is not None:
            c.set_path(path)
        out.append(c)
        x0 += X
    G.comm_init_local(out)
    return out


def _whole(G, X, Y, Z, seed, path=None, bs=2):
    import gcm_amd
    U, U1, L = _mats()
    c = gcm_amd.Context(3, bs, [X, Y, Z])
    c.set_materials(U[None], U1[None], L[None])
    c.fill_random([X, Y, Z], seed)
    if path is not None:
        c.set_path(path)
    return c


def _inner(c, arr, bs=2):
    return arr.reshape(tuple(s + 2 * bs for s in c.sizes) + (9,))[bs:-bs, bs:-bs, bs:-bs]


def _concat(slabs, bs=2):
    return np.concatenate([_inner(c, c.download(), bs) for c in slabs], axis=0)


def _run_threads(fns):
    """One host thread per rank, as RCCL ranks run (ctypes releases the GIL)."""
    errs = [None] * len(fns)

    def go(i):
        try:
            fns[i]()
        except Exception as e:  # reported below
            errs[i] = e
    th = [threading.Thread(target=go, args=(i,)) for i in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in errs:
        if e is not None:
            raise e


@pytest.mark.parametrize("sched", ["auto", "single", "xslab", "bfirst"])
@pytest.mark.parametrize("xs", [[17, 23], [12, 9, 19], [8, 6, 10], [9, 6, 7]])
def test_local_group_fused_equals_whole(G, sched, xs):
    """Ragged slabs on the fused path: the X-slab schedule (auto: a configured
    exchange selects it) with the in-step overlapped exchange, and the one-launch
    schedule with the exchange in front; 4 steps == one context, bitwise."""
    Y, Z, seed, steps = 40, 64, 0x5EED, 4
    sc = {"auto": None, "single": G.SCHED_SINGLE, "xslab": G.SCHED_XSLAB, "bfirst": G.SCHED_BFIRST}[sched]
    slabs = _group(G, xs, Y, Z, seed, sched=sc)
    whole = _whole(G, sum(xs), Y, Z, seed)
    G.local_group_steps(slabs, 0.9, steps)
    for _ in range(steps):
        whole.step(0.9)
    assert all(c.last_path == "fused" for c in slabs)
    want = _inner(whole, whole.download())
    assert np.array_equal(_concat(slabs), want)
    for c in slabs + [whole]:
        c.close()


@pytest.mark.parametrize("sched", ["xslab", "bfirst"])
def test_local_group_zsplit_rows_equal_whole(G, sched):
    """Rows of 1024 nodes (the z-split step, k_step_tx2<..., ZS> + k_zseam, on
    plane ranges and the boundary-first two-range launch) in a ragged slab group
    == one context, bitwise."""
    xs, Y, Z, seed, steps = [9, 6, 7], 10, 1024, 0x5EED, 3
    sc = {"xslab": G.SCHED_XSLAB, "bfirst": G.SCHED_BFIRST}[sched]
    slabs = _group(G, xs, Y, Z, seed, sched=sc)
    whole = _whole(G, sum(xs), Y, Z, seed)
    for c in slabs + [whole]:
        c.profile(True)
    G.local_group_steps(slabs, 0.9, steps)
    for _ in range(steps):
        whole.step(0.9)
    assert all(c.last_path == "fused" for c in slabs)
    assert "ZS" in whole.profile_read()["fused_xyz"]["kernel"]
    assert np.array_equal(_concat(slabs), _inner(whole, whole.download()))
    for c in slabs + [whole]:
        c.close()


def test_local_group_split_path_per_stage_exchange(G):
    """Split path (gcmx_stage per axis): the X stage's halo is exchanged inside
    stage(0) (halo_ensure), per stage, as gcmx_stage with a communicator does."""
    xs, Y, Z, seed, steps = [10, 14, 8], 24, 40, 0x5EED, 3
    slabs = _group(G, xs, Y, Z, seed, path=G.PATH_SPLIT)
    whole = _whole(G, sum(xs), Y, Z, seed, path=G.PATH_SPLIT)

    def stepper(c):
        def f():
            for _ in range(steps):
                for s in range(3):
                    c.stage(s, 0.9)
            c.sync()
        return f
    _run_threads([stepper(c) for c in slabs])
    for _ in range(steps):
        for s in range(3):
            whole.stage(s, 0.9)
    assert all(c.last_path == "split" for c in slabs)
    assert np.array_equal(_concat(slabs), _inner(whole, whole.download()))
    for c in slabs + [whole]:
        c.close()


@pytest.mark.parametrize("path", ["fused", "split"])
def test_local_group_with_x_faces(G, path):
    """Free-surface and force conditions on all six faces (gcmx_step_faces): the
    x faces belong to the outer slabs only, the inner X boundaries are halos; the
    fused path forms the y/z face ghosts in the one pass, the split path fills
    every face per stage and exchanges the halo inside stage(0)."""
    xs, Y, Z, seed, steps = [11, 13], 30, 48, 0x5EED, 3
    p = G.PATH_FUSED if path == "fused" else G.PATH_SPLIT
    slabs = _group(G, xs, Y, Z, seed, path=p)
    whole = _whole(G, sum(xs), Y, Z, seed, path=p)
    q = G.QUANTITY_CODES
    free = [(q["Sxx"], 0.0), (q["Sxy"], 0.0), (q["Sxz"], 0.0)]
    pull = [(q["Syy"], -0.25), (q["Syz"], 0.0)]
    faces_all = [free, free, pull, pull, [(q["Vz"], 0.0)], [(q["Szz"], 0.5)]]

    def faces_for(r):
        f = list(faces_all)
        if r > 0:
            f[0] = None
        if r < len(xs) - 1:
            f[1] = None
        return f

    def stepper(r, c):
        def f():
            for _ in range(steps):
                c.step_faces(0.9, faces_for(r))
            c.sync()
        return f
    _run_threads([stepper(r, c) for r, c in enumerate(slabs)])
    for _ in range(steps):
        whole.step_faces(0.9, faces_all)
    assert whole.last_path == path and all(c.last_path == path for c in slabs)
    assert np.array_equal(_concat(slabs), _inner(whole, whole.download()))
    for c in slabs + [whole]:
        c.close()


@pytest.mark.timeout(60)
def test_local_group_unpaired_rank_times_out(G, monkeypatch):
    """A rank whose neighbour never steps fails with GCMX_ERR_COMM (the wait is
    bounded) instead of reading stale ghosts."""
    monkeypatch.setenv("GCMX_LOCAL_WAIT_SECONDS", "2")
    slabs = _group(G, [8, 8], 16, 32, 1)
    with pytest.raises(G.GcmxError) as ei:
        slabs[0].step(0.9)
    assert ei.value.status == 7  # GCMX_ERR_COMM
    for c in slabs:
        c.close()


def _oracle_steps(X, Y, Z, seed, steps):
    b = oracle_body(3, 2, [X, Y, Z])
    O.fill_random(b, [X, Y, Z], seed)
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or len(os.sched_getaffinity(0))
    for _ in range(steps):
        for s in range(3):
            b.stage(s, 0.9, threads)
    return b.inner_view()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("sched", ["xslab", "bfirst"])
def test_local_group_two_64x512x512_slabs_match_oracle(G, sched):
    """Config 3's slab shape (512^3 over 8 GPUs = 64 x 512 x 512 per rank): two
    such ranks in one group, 2 steps with the overlapped in-step exchange
    (three-stream and boundary-first schedules), == the oracle on the undivided
    128 x 512 x 512 box, bitwise."""
    X, Y, Z, seed, steps = 64, 512, 512, 0x5EED, 2
    slabs = _group(G, [X, X], Y, Z, seed, sched={"xslab": G.SCHED_XSLAB, "bfirst": G.SCHED_BFIRST}[sched])
    G.local_group_steps(slabs, 0.9, steps)
    assert all(c.last_path == "fused" for c in slabs)
    got = _concat(slabs)
    for c in slabs:
        c.close()
    assert np.array_equal(got, _oracle_steps(2 * X, Y, Z, seed, steps))


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_local_group_eight_slabs_whole_512_match_oracle(G):
    """The whole config-3 decomposition on one device: 512^3 as eight 64 x 512
    x 512 ranks (about 22 GB of layers), 2 steps with the overlapped in-step
    exchange, == the oracle on the undivided 512^3 grid, bitwise."""
    X, N, seed, steps = 64, 512, 0x5EED, 2
    slabs = _group(G, [X] * 8, N, N, seed)
    G.local_group_steps(slabs, 0.9, steps)
    assert all(c.last_path == "fused" for c in slabs)
    got = _concat(slabs)
    for c in slabs:
        c.close()
    want = _oracle_steps(N, N, N, seed, steps)
    for r in range(8):
        assert np.array_equal(got[r * X:(r + 1) * X], want[r * X:(r + 1) * X]), f"slab {r}"


@pytest.mark.parametrize("sched", ["auto", "xslab", "single"])
def test_loopback_exchange_is_periodic_halo(G, sched):
    """The loopback transport (gcmx_comm_init_loopback: one slab exchanging with
    itself through the RCCL post / wait points, held at an emulated link rate)
    fills the x ghosts periodically: 3 fused steps == the per-stage path with
    the same periodic ghosts written by gcmx_copy_box before each step,
    bitwise."""
    X, Y, Z, seed, steps = 18, 24, 64, 0x5EED, 3
    a = _whole(G, X, Y, Z, seed)
    if sched != "auto":
        a.set_schedule({"xslab": G.SCHED_XSLAB, "single": G.SCHED_SINGLE}[sched])
    a.comm_init_loopback(64.0, 4)
    b = _whole(G, X, Y, Z, seed, path=G.PATH_SPLIT)  # an independent path: per-stage kernels
    for _ in range(steps):
        a.step(0.9)
        b.copy_box([-2, 0, 0], [0, Y, Z], b, [X - 2, 0, 0])
        b.copy_box([X, 0, 0], [X + 2, Y, Z], b, [0, 0, 0])
        b.step(0.9)
    a.sync()
    assert a.last_path == "fused" and b.last_path == "split"
    assert np.array_equal(_inner(a, a.download()), _inner(b, b.download()))
    for c in (a, b):
        c.close()


def test_rccl_single_rank_communicator(G):
    """gcmx_comm_init on this box's RCCL (ncclCommInitRankConfig with the
    minCTAs request): a one-rank communicator has no neighbours, so the step
    runs without an exchange and equals a context without a communicator."""
    import gcm_amd
    X, Y, Z, seed = 16, 24, 64, 0x5EED
    a = _whole(G, X, Y, Z, seed)
    a.comm_init(gcm_amd.unique_id(), 1, 0, -1, -1)
    b = _whole(G, X, Y, Z, seed, path=G.PATH_SPLIT)  # an independent path: per-stage kernels
    for _ in range(2):
        a.step(0.9)
        b.step(0.9)
    assert a.last_path == "fused"
    assert np.array_equal(a.download(), b.download())
    for c in (a, b):
        c.close()


@pytest.mark.parametrize("sched", ["auto", "xslab", "single", "split"])
def test_rccl_self_exchange(G, sched):
    """The REAL RCCL exchange on one GPU: a one-rank communicator whose left and
    right neighbours are itself (gcmx_comm_init(.., 1, 0, 0, 0)), so every post
    point runs the ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd group and
    the ev_halo ordering an N > 1 rank runs.  RCCL pairs a rank's sends to itself
    with its receives in posting order: the left ghosts receive the first two
    inner planes, the right ghosts the last two.  3 steps (the boundary-first,
    X-slab and one-launch schedules, and the split path's per-stage exchange) ==
    the per-stage path with those ghosts written by gcmx_copy_box, bitwise."""
    import gcm_amd
    X, Y, Z, seed, steps = 18, 24, 64, 0x5EED, 3
    a = _whole(G, X, Y, Z, seed)
    if sched == "split":
        a.set_path(G.PATH_SPLIT)
    elif sched != "auto":
        a.set_schedule({"xslab": G.SCHED_XSLAB, "single": G.SCHED_SINGLE}[sched])
    a.comm_init(gcm_amd.unique_id(), 1, 0, 0, 0)
    b = _whole(G, X, Y, Z, seed, path=G.PATH_SPLIT)  # an independent path: per-stage kernels
    for _ in range(steps):
        a.step(0.9)
        b.copy_box([-2, 0, 0], [0, Y, Z], b, [0, 0, 0])
        b.copy_box([X, 0, 0], [X + 2, Y, Z], b, [X - 2, 0, 0])
        b.step(0.9)
    a.sync()
    assert a.last_path == ("split" if sched == "split" else "fused") and b.last_path == "split"
    assert np.array_equal(_inner(a, a.download()), _inner(b, b.download()))
    for c in (a, b):
        c.close()


@pytest.mark.timeout(200)
def test_rccl_self_exchange_on_shuffled_layers(G):
    """The same RCCL self-exchange on layers large enough for the default
    shuffled physical-chunk mapping (435 MB, 64 MiB chunks): RCCL
    sends from and receives into the mapped range; 2 steps == the per-stage path
    with copied ghosts, bitwise."""
    import gcm_amd
    X, Y, Z, seed, steps = 18, 256, 512, 0x5EED, 2
    a = _whole(G, X, Y, Z, seed)
    info = a.layer_info()
    if "GCMX_ALLOC" not in __import__("os").environ:
        assert info["alloc"] == "shuffled 64 MiB chunks", info
    a.comm_init(gcm_amd.unique_id(), 1, 0, 0, 0)
    b = _whole(G, X, Y, Z, seed, path=G.PATH_SPLIT)
    for _ in range(steps):
        a.step(0.9)
        b.copy_box([-2, 0, 0], [0, Y, Z], b, [0, 0, 0])
        b.copy_box([X, 0, 0], [X + 2, Y, Z], b, [X - 2, 0, 0])
        b.step(0.9)
    a.sync()
    assert a.last_path == "fused"
    assert np.array_equal(_inner(a, a.download()), _inner(b, b.download()))
    for c in (a, b):
        c.close()


@pytest.mark.timeout(120)
def test_rccl_stalled_exchange_fails_instead_of_hanging(G):
    """VERDICT r3 item 6 (the reference's analogue is the blocking
    MPI_Sendrecv_replace of TestMPI.cpp:33-50): a peer that never posts must not
    hang the rank.  A one-rank self-communicator whose exchange groups post their
    sends but never their receives (gcmx_comm_test_stall) cannot complete an
    exchange; the non-blocking communicator's bounded waits then abort it and
    gcmx_sync returns GCMX_ERR_COMM within the timeout, and every later step of
    the context fails with GCMX_ERR_COMM too."""
    import time
    import gcm_amd
    X, Y, Z, seed = 18, 24, 64, 0x5EED
    a = _whole(G, X, Y, Z, seed)
    a.comm_init(gcm_amd.unique_id(), 1, 0, 0, 0, timeout_s=5.0)
    a.comm_test_stall(True)
    t0 = time.time()
    with pytest.raises(gcm_amd.GcmxError) as e:
        for _ in range(2):
            a.step(0.9)
        a.sync()
    assert e.value.status == 7, str(e.value)  # GCMX_ERR_COMM
    assert time.time() - t0 < 60
    with pytest.raises(gcm_amd.GcmxError) as e2:
        a.step(0.9)
        a.sync()
    assert e2.value.status == 7
    a.close()


def test_rccl_channels_fixed_per_process_is_checked(G):
    """RCCL reads NCCL_NCHANNELS_PER_PEER once per process,
    so the library fixes the count at the process's first communicator and
    REFUSES (GCMX_ERR_STATE, before any RCCL call) a later communicator that
    needs another count, instead of letting it run silently with the first
    one's; asking for the fixed count explicitly works."""
    import gcm_amd
    a = _whole(G, 8, 24, 64, 1)
    a.comm_init(gcm_amd.unique_id(), 1, 0, -1, -1)
    fixed = a.comm_channels_per_peer
    assert fixed >= 0
    b = _whole(G, 8, 24, 64, 1)
    with pytest.raises(gcm_amd.GcmxError) as e:
        b.comm_init(gcm_amd.unique_id(), 1, 0, -1, -1, channels_per_peer=fixed + 1)
    assert e.value.status == 5 and "fixed" in str(e.value), str(e.value)  # GCMX_ERR_STATE
    b.comm_init(gcm_amd.unique_id(), 1, 0, -1, -1, channels_per_peer=fixed)
    assert b.comm_channels_per_peer == fixed
    for c in (a, b):
        c.close()


def test_rccl_self_exchange_timings(G):
    """the exchange is timed.  A one-rank self-exchange (the
    real ncclSend / ncclRecv group every step) with profiling on: every post is
    one `halo_rccl` bucket entry (comm stream, data-ready -> last kernel) whose
    bytes are what one link direction carries, every wait of the compute stream
    one `halo_wait` entry, and bench.py's rank_record turns them into the
    per_rank fields of an N > 1 line.  Every group posted all its calls."""
    import gcm_amd
    import bench
    X, Y, Z, steps = 16, 24, 64, 6
    a = _whole(G, X, Y, Z, 0x5EED)
    a.comm_init(gcm_amd.unique_id(), 1, 0, 0, 0)
    a.step(0.9)
    a.sync()
    calls0 = a.comm_posted_calls
    a.profile(True)
    a.profile_reset()
    for _ in range(steps):
        a.step(0.9)
    a.sync()
    k = a.profile_read()
    a.profile(False)
    assert "halo_rccl" in k and "halo_wait" in k, sorted(k)
    assert k["halo_rccl"]["launches"] == steps
    comps = 6  # the X stage reads 6 of the 9 components at its neighbours
    plane = (Y + 4) * (((2 + 14) + Z + 2 + 15) // 16 * 16)  # ghost-padded y rows x padded z row
    assert k["halo_rccl"]["bytes_per_launch"] == 8.0 * 2 * plane * comps
    rec = bench.rank_record(a, 0, k, steps, 1.0)
    assert rec["halo_ms"] > 0 and rec["GBps_per_direction"] > 0
    assert rec["halo_posts_per_step"] == 1.0 and rec["transport"] == "halo_rccl"
    assert rec["exposed_wait_ms"] >= 0 and rec["interior_ms"] > 0 and rec["boundary_ms"] > 0
    assert rec["channels_per_peer"] == a.comm_channels_per_peer
    # every group: a send and a receive per halo component and neighbour (left = right = self)
    assert a.comm_posted_calls - calls0 == steps * comps * 2 * 2
    a.close()


def test_rccl_self_neighbour_needs_one_rank(G):
    """A neighbour equal to the rank itself is refused in a multi-rank communicator."""
    import gcm_amd
    a = _whole(G, 8, 16, 32, 1)
    with pytest.raises(gcm_amd.GcmxError):
        a.comm_init(gcm_amd.unique_id(), 2, 0, 0, 1)
    a.close()


@pytest.mark.parametrize("sched", ["bfirst", "xslab"])
@pytest.mark.parametrize("xs", [[4, 7, 5], [9, 6]])
def test_local_group_border_size_one(G, sched, xs):
    """borderSize 1: each boundary side is ONE plane, so the boundary-first
    schedule's two-range launch covers two odd ranges (each pair's second plane
    clamped and not stored); 3 steps == one context, bitwise."""
    Y, Z, seed, steps, bs = 20, 64, 0x5EED, 3, 1
    sc = {"xslab": G.SCHED_XSLAB, "bfirst": G.SCHED_BFIRST}[sched]
    slabs = _group(G, xs, Y, Z, seed, sched=sc, bs=bs)
    whole = _whole(G, sum(xs), Y, Z, seed, bs=bs)
    G.local_group_steps(slabs, 0.9, steps)
    for _ in range(steps):
        whole.step(0.9)
    assert all(c.last_path == "fused" for c in slabs)
    assert np.array_equal(_concat(slabs, bs), _inner(whole, whole.download(), bs))
    for c in slabs + [whole]:
        c.close()


@pytest.mark.parametrize("ids_on", [(True, False, True), (True, True, True), (False, True, False)])
def test_local_group_step_ode_mixed_material_ids(G, monkeypatch, ids_on):
    """gcmx_step_ode on slabs where only some ranks carry per-node
    material ids.  Those ranks run the separate ODE pass (not folded), the
    others fold it into the one-pass step; every rank must still post its halo
    exactly once per step (the in-step post only when the step's result is
    final), else the in-process group pairs the wrong generations and times
    out -- RCCL would hang.  Equal, bitwise, to one context with the same ids."""
    import gcm_amd
    monkeypatch.setenv("GCMX_LOCAL_WAIT_SECONDS", "20")
    U, U1, L = _mats()
    from gcm_amd.host import isotropic_elastic_matrices
    U2, U12, L2 = isotropic_elastic_matrices(3, 2.5, 2.0, 1.0)
    Um, U1m, Lm = np.stack([U, U2]), np.stack([U1, U12]), np.stack([L, L2])
    xs, Y, Z, seed, steps, bs = [8, 7, 9], 12, 64, 0x5EED, 3, 2
    Xg = sum(xs)
    tau = 0.9 / np.sqrt(8.0 / 4.0)  # Courant 0.9 of the faster material (c1 = sqrt(8/4))
    # global ids: material 1 in the slabs that carry ids, at z >= 32
    def ids_for(sizes, on):
        ids = np.zeros(tuple(s + 2 * bs for s in sizes), dtype=np.uint8)
        if on:
            ids[:, :, bs + 32:] = 1
        return ids
    slabs, x0 = [], 0
    for X, on in zip(xs, ids_on):
        c = gcm_amd.Context(3, bs, [X, Y, Z], start=[x0, 0, 0])
        if on:
            c.set_materials(Um, U1m, Lm)
            c.set_material_ids(ids_for([X, Y, Z], True).reshape(-1))
        else:
            c.set_materials(U[None], U1[None], L[None])
        c.fill_random([Xg, Y, Z], seed)
        slabs.append(c)
        x0 += X
    G.comm_init_local(slabs)
    tau0 = {True: [3.0, 2.0], False: [3.0]}

    def rank(i):
        def go():
            for _ in range(steps):
                slabs[i].step_ode(tau, tau0[ids_on[i]])
            slabs[i].sync()
        return go
    _run_threads([rank(i) for i in range(len(xs))])
    got = _concat(slabs)
    # the same grid as one context: ids where a slab carries them
    w = gcm_amd.Context(3, bs, [Xg, Y, Z])
    w.set_materials(Um, U1m, Lm)
    gid = np.zeros((Xg + 2 * bs, Y + 2 * bs, Z + 2 * bs), dtype=np.uint8)
    x0 = 0
    for X, on in zip(xs, ids_on):
        if on:
            gid[bs + x0:bs + x0 + X, :, bs + 32:] = 1
        x0 += X
    w.set_material_ids(gid.reshape(-1))
    w.fill_random([Xg, Y, Z], seed)
    for _ in range(steps):
        w.step_ode(tau, [3.0, 2.0])
    assert np.array_equal(got, _inner(w, w.download()))
    for c in slabs + [w]:
        c.close()
