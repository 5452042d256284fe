#!/usr/bin/env python3
"""Per-GPU time of one X slab of the 512^3 strong-scaling run, on ONE GPU.

For each slab thickness X (512 / N for N = 1, 2, 4, 8) a [X, 512, 512] context
runs the fused step under a multi-GPU step schedule (gcmx_set_step_schedule):
bfirst (default; what a rank runs: both boundary sides in one launch of thin
blocks, then the interior on the same stream), xslab (interior on a
low-priority stream beside 16-row boundary blocks) or single (one launch).
With --loop-gbps R the slab also exchanges its halo -- with itself, through the
loopback transport (gcmx_comm_init_loopback) at the RCCL post / wait points,
each transfer holding a few CU slots for the time its bytes take at R GB/s per
direction -- so the time is one rank's step with the exchange in flight;
without it the transfers are not emulated.  With --rccl-self the slab is a
one-rank RCCL communicator whose neighbours are itself (gcmx_comm_init, left =
right = 0): the real ncclSend/ncclRecv group runs at every post point, its
bytes moved by RCCL's own kernels on the same GPU.  --rows sets the interior's y rows
per block (0: automatic).  Also checks the slab step bitwise against the
generic per-stage path on a [64, 512, 512] slab.  One JSON line per size.

    python scripts/bench_slab.py [--sched bfirst|xslab|single] [--loop-gbps R] [--ranks 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import gcm_amd  # noqa: E402
from gcm_amd import gcmx  # noqa: E402
from gcm_amd.host import isotropic_elastic_matrices  # noqa: E402
from bench import rank_record, stdout_to_stderr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sched", default="bfirst", choices=["single", "xslab", "bfirst"])
ap.add_argument("--loop-gbps", type=float, default=-1.0,
                help=">= 0: loopback transport (gcmx_comm_init_loopback): the slab exchanges "
                     "with itself through the RCCL post/wait points, held for the bytes' time "
                     "at this rate per direction (xGMI emulation); < 0: no exchange")
ap.add_argument("--loop-blocks", type=int, default=128)
ap.add_argument("--rccl-self", action="store_true",
                help="one-rank RCCL communicator exchanging with itself (real ncclSend/Recv)")
ap.add_argument("--rows", type=int, default=0)
ap.add_argument("--ranks", default="1,2,4,8")
ap.add_argument("--n", type=int, default=512)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--no-check", action="store_true")
ap.add_argument("--reps", type=int, default=5, help="timed repetitions of --steps steps (median)")
args = ap.parse_args()
if args.rccl_self and len(args.ranks.split(",")) > 1:
    # RCCL reads NCCL_NCHANNELS_PER_PEER once per process: the first
    # communicator fixes the channel count, and the library refuses a later one
    # that needs another (gcmx.h, checked contract).  One process per rank count.
    sys.exit("--rccl-self: give one --ranks value per process (RCCL fixes the channel count per process)")
U, U1, L = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
N, STEPS = args.n, args.steps
SCHED = {"xslab": gcmx.SCHED_XSLAB, "bfirst": gcmx.SCHED_BFIRST}.get(args.sched, gcmx.SCHED_SINGLE)


def make(X, path=gcmx.PATH_AUTO, x0=0, loop=False):
    c = gcm_amd.Context(3, 2, [X, N, N], start=[x0, 0, 0], device=0)
    c.set_materials(U[None], U1[None], L[None])
    c.set_path(path)
    c.set_schedule(SCHED, args.rows)
    c.fill_random([N, N, N], 0x5EED)
    if loop and args.rccl_self:
        with stdout_to_stderr():  # RCCL's banner stays off the JSON lines
            c.comm_init(gcm_amd.unique_id(), 1, 0, 0, 0)
    elif loop and args.loop_gbps >= 0:
        c.comm_init_loopback(args.loop_gbps, args.loop_blocks)
    return c


if not args.no_check:
    outs = {}
    for name, path in (("fused", gcmx.PATH_FUSED), ("generic", gcmx.PATH_GENERIC)):
        c = make(64, path, x0=128)
        c.fp_mode = gcmx.FP_EXACT  # the schedule's check is bitwise: the exact build of the step
        for _ in range(2):
            c.step(0.9)
        outs[name] = c.download()
        c.close()
    bad = int(np.sum(outs["fused"] != outs["generic"]))
    print(json.dumps({"check": "slab 64x512x512 fused (exact fp build) vs generic, 2 steps", "mismatches": bad,
                      "sched": args.sched, "rows": args.rows,
                      "boundary_rows": os.environ.get("GCMX_BOUNDARY_ROWS", "default")}), flush=True)
    if bad:
        sys.exit(1)

for ranks in [int(r) for r in args.ranks.split(",")]:
    X = N // ranks
    c = make(X, loop=True)
    for _ in range(3):
        c.step(0.9)
    c.sync()
    reps = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        for _ in range(STEPS):
            c.step(0.9)
        c.sync()
        reps.append(time.perf_counter() - t0)
    el = sorted(reps)[len(reps) // 2]
    c.profile(True)
    c.profile_reset()
    for _ in range(STEPS):
        c.step(0.9)
    c.sync()
    k = c.profile_read()
    c.profile(False)
    # the exchange / compute split of this rank (bench.py rank_record): halo_ms,
    # exposed_wait_ms, bytes and GB/s per direction, channels per peer
    rec = rank_record(c, 0, k, STEPS, el / STEPS * 1e3) if (args.rccl_self or args.loop_gbps >= 0) else None
    c.close()
    ms = el / STEPS * 1e3
    rate = X * N * N * STEPS / el / 1e6
    kern = {n: round(v["total_ms"] / max(1, v["launches"]), 4) for n, v in k.items()}
    ksum = sum(v["total_ms"] for v in k.values()) / STEPS
    print(json.dumps({"ranks": ranks, "slab": [X, N, N], "ms_per_step": round(ms, 4),
                      "rep_ms_per_step": [round(r / STEPS * 1e3, 4) for r in reps],
                      "kernel_ms_per_step": round(ksum, 4),
                      "Mnode_steps_per_gpu": round(rate, 1),
                      "projected_job_rate": round(rate * ranks, 1),
                      "kernels": kern,
                      "per_rank": [rec] if rec else None,
                      "sched": args.sched, "rows": args.rows,
                      "boundary_rows": os.environ.get("GCMX_BOUNDARY_ROWS", "default"),
                      "exchange": "RCCL self-exchange (one-rank communicator)" if args.rccl_self else
                                  (f"loopback {args.loop_gbps} GB/s per direction, "
                                   f"{args.loop_blocks} blocks" if args.loop_gbps >= 0 else
                                   "none (transfers not emulated)")}), flush=True)
