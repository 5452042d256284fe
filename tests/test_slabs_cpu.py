"""Multi-rank X-slab decomposition on CPU (gloo, world_size 2 and 3).

Each rank owns an X slab of a 3-D grid (the layout bench.py / gcmx_comm_init use)
and, before every time step, exchanges its first/last borderSize inner x-planes
with its neighbours into their ghost planes (the halo gcmx_halo_exchange sends
over RCCL).  The stage numerics are the oracle's.  Every rank's slab must be
bitwise equal to the same region of a single-domain run (the
Engine.AdhesionContact property, TestEngine.cpp:27-87)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _slab_bounds(N, world, rank):
    """bench.py's partition: equal slabs (N divisible by world) or remainder on the last."""
    X = N // world
    x0 = rank * X
    return x0, (N - x0 if rank == world - 1 else X)


def _worker(rank, world, port, N, bs, steps, halo_comps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import oracle as O
        from tests.helpers import oracle_body
        x0, X = _slab_bounds(N, world, rank)
        b = oracle_body(3, bs, [X, N, N], start=[x0, 0, 0])
        O.fill_random(b, [N, N, N], 0x5EED)
        full = oracle_body(3, bs, [N, N, N])
        O.fill_random(full, [N, N, N], 0x5EED)
        left = rank - 1 if rank > 0 else -1
        right = rank + 1 if rank < world - 1 else -1
        for _ in range(steps):
            cur = b.pde.reshape(b.shape_all + (9,))
            reqs = []
            bufs = []
            for c in halo_comps:
                if left >= 0:
                    send = torch.from_numpy(np.ascontiguousarray(cur[bs:2 * bs, :, :, c]))
                    recv = torch.empty_like(send)
                    reqs += [dist.isend(send, left), dist.irecv(recv, left)]
                    bufs.append((recv, slice(0, bs), c))
                if right >= 0:
                    send = torch.from_numpy(np.ascontiguousarray(cur[X:X + bs, :, :, c]))
                    recv = torch.empty_like(send)
                    reqs += [dist.isend(send, right), dist.irecv(recv, right)]
                    bufs.append((recv, slice(X + bs, X + 2 * bs), c))
            for r in reqs:
                r.wait()
            for recv, sl, c in bufs:
                cur[sl, :, :, c] = recv.numpy()
            for s in range(3):
                b.stage(s, 0.9)
            for s in range(3):
                full.stage(s, 0.9)
        mine = b.inner_view()
        ref = full.inner_view()[x0:x0 + X]
        q.put((rank, bool(np.array_equal(mine, ref)), int(np.sum(mine != ref))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 16), (3, 17)])
def test_x_slabs_gloo_bitwise(world, N):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    halo = [0, 1, 2, 3, 4, 5]  # components the X stage reads at its neighbours
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, 2, 3, halo, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, bad in sorted(res):
        assert ok, f"rank {rank}: {bad} values differ from the single-domain run"


def test_halo_components_are_what_the_x_stage_reads():
    """The halo carries exactly the components with a non-zero U entry in a row
    with a non-zero eigenvalue along X (gcmx compute_halo_comps)."""
    from oracle import oracle as O
    U, U1, L = O.isotropic_elastic_matrices(3, 4, 2, 1)
    need = sorted({j for k in range(9) if L[0, k] != 0 for j in range(9) if U[0, k, j] != 0})
    assert need == [0, 1, 2, 3, 4, 5]
