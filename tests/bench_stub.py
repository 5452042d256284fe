"""Test stand-in for gcm_amd in bench.py (GCM_BENCH_BACKEND=tests.bench_stub).

TEST INFRASTRUCTURE ONLY: it lets bench.py's N > 1 orchestration -- the ranks it
starts itself, the unique-id broadcast, the comm_init arguments, the MAX of the
repetition times over ranks, the per_rank gather, multi_gpu_parity's slab
concatenation -- run under gloo on the CPU.  A `Context` is an oracle Body
(oracle/, the CPU restatement of the reference stage, GridCharacteristicMethod.hpp:42-52);
after comm_init every step first swaps the borderSize x planes with the
neighbour ranks over the default (gloo) process group, as the reference's
MPI_Sendrecv_replace X-slab exchange does (src/test/TestMPI.cpp:33-47), then runs
the three stages.  Every call the orchestration makes is logged and written to
$GCM_BENCH_STUB_LOG/rank<r>.json when the process exits.
"""
import atexit
import json
import os
import sys
import time
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from tests.helpers import oracle_body  # noqa: E402

_RANK = int(os.environ.get("RANK", "0"))
_LOG = {"rank": _RANK, "world": int(os.environ.get("WORLD_SIZE", "1")), "unique_ids": [],
        "contexts": [], "comm_init": [], "exchanges": 0, "pid": os.getpid()}


def _dump():
    d = os.environ.get("GCM_BENCH_STUB_LOG")
    if d:
        with open(os.path.join(d, f"rank{_RANK}.json"), "w") as f:
            json.dump(_LOG, f)


atexit.register(_dump)


def unique_id() -> bytes:
    uid = os.urandom(128)  # the size of an ncclUniqueId
    _LOG["unique_ids"].append(uid.hex())
    return uid


class Context:
    def __init__(self, dim, border_size, sizes, start=None, device=0):
        self.bs = border_size
        self.sizes = list(sizes)
        self.start = list(start) if start is not None else [0] * dim
        self.body = oracle_body(dim, border_size, sizes, start=self.start)
        self.body.pde[:] = 0.0
        self.comm = None
        self.prof = False
        self.buckets = {}
        self.fp_mode = 0
        self.comm_channels_per_peer = 0
        _LOG["contexts"].append({"sizes": self.sizes, "start": self.start, "device": device})

    # --- set-up ---
    def layer_info(self):
        return {"a": 0x1000, "b": 0x2000, "layer_bytes": self.body.pde.nbytes, "one_allocation": True,
                "alloc": "stub"}

    def set_materials(self, U, U1, L):
        pass

    def set_path(self, path):
        pass

    def set_schedule(self, sched, rows_per_block=0):
        pass

    def fill_random(self, global_sizes, seed):
        O.fill_random(self.body, global_sizes, seed)

    def comm_init(self, uid, nranks, rank, left, right, global_x=None, channels_per_peer=0):
        _LOG["comm_init"].append({"uid": uid.hex(), "nranks": nranks, "rank": rank, "left": left,
                                  "right": right, "global_x": global_x,
                                  "channels_per_peer": channels_per_peer, "sizes": self.sizes,
                                  "start": self.start})
        self.comm = (left, right)
        self.comm_channels_per_peer = channels_per_peer or 4

    @property
    def effective_path(self):
        return "stub-oracle"

    last_path = effective_path

    @property
    def device_bytes(self):
        return 2 * self.body.pde.nbytes

    # --- the step ---
    def _exchange(self):
        import torch
        import torch.distributed as dist
        bs, X = self.bs, self.sizes[0]
        cur = self.body.pde.reshape(self.body.shape_all + (self.body.M,))
        reqs, bufs = [], []
        for nb, send_sl, recv_sl in ((self.comm[0], slice(bs, 2 * bs), slice(0, bs)),
                                     (self.comm[1], slice(X, X + bs), slice(X + bs, X + 2 * bs))):
            if nb < 0:
                continue
            send = torch.from_numpy(np.ascontiguousarray(cur[send_sl]))
            recv = torch.empty_like(send)
            reqs += [dist.isend(send, nb), dist.irecv(recv, nb)]
            bufs.append((recv, recv_sl))
        for r in reqs:
            r.wait()
        for recv, sl in bufs:
            cur[sl] = recv.numpy()
        _LOG["exchanges"] += 1
        return sum(b[0].numel() for b in bufs) * 8 // max(1, len(bufs))

    def _add(self, name, ms, nbytes, kernel):
        if self.prof:
            b = self.buckets.setdefault(name, {"total_ms": 0.0, "launches": 0, "kernel": kernel,
                                               "bytes_per_launch": nbytes})
            b["total_ms"] += ms
            b["launches"] += 1

    def step(self, tau):
        if os.environ.get("GCM_BENCH_STUB_FAIL_RANK") == str(_RANK):
            raise RuntimeError("stub: this rank fails (GCM_BENCH_STUB_FAIL_RANK)")
        t0 = time.perf_counter()
        if self.comm is not None:
            nb = 0 if os.environ.get("GCM_BENCH_STUB_NO_EXCHANGE") else self._exchange()
            self._add("halo_rccl", (time.perf_counter() - t0) * 1e3, nb, "stub gloo exchange")
            self._add("halo_wait", 0.0, 0, "stub")
        t1 = time.perf_counter()
        for s in range(3):
            self.body.stage(s, tau)
        n = int(np.prod(self.sizes))
        self._add("fused_xyz", (time.perf_counter() - t1) * 1e3, 144 * n, "stub oracle stages")

    def sync(self):
        pass

    def download(self):
        return self.body.pde.copy()

    # --- measurement hooks ---
    def profile(self, on=True):
        self.prof = on

    def profile_reset(self):
        self.buckets = {}

    def profile_read(self):
        return {k: dict(v) for k, v in self.buckets.items()}

    def close(self):
        pass


gcmx = types.SimpleNamespace(PATH_AUTO=0, PATH_GENERIC=1, PATH_SPLIT=2, PATH_FUSED=3, SCHED_AUTO=0,
                             FP_EXACT=1, FP_FMA=0, LIB_PATH=os.path.abspath(__file__))
gcm_amd = types.SimpleNamespace(Context=Context, unique_id=unique_id, gcmx=gcmx)
