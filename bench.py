#!/usr/bin/env python3
"""Headline benchmark: 3-D isotropic-elastic CubicGrid stage loop, 512^3, fp64.

One step = one full time step of cubic::Engine::nextTimeStep (all three stages,
engine/cubic/Engine.cpp:90-121) over the whole grid, inputs resident in HBM.
`python bench.py --gpus N --steps K --warmup W`; for N > 1 the 512^3 grid is
split into N X-slabs, one rank per GPU, with an RCCL halo exchange of the X
ghost planes every step (strong scaling: the total work is fixed).  The ranks
come from a launcher (torch.distributed.run sets RANK / WORLD_SIZE / ...) or,
when none set WORLD_SIZE, from bench.py itself: the parent process counts the
devices (no GPU call), starts N rank processes with the launcher's variables
and relays rank 0's JSON line (`self_launch`).

Prints ONE JSON line on rank 0 (see README/DESIGN for the fields).
"""
import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tools import box_state  # noqa: E402  (read-only amdgpu sysfs, measurement context)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
BYTES_PER_NODE_STAGE = 2 * 9 * 8  # read + write the 9-component fp64 state
JSON_OUT = sys.stdout  # main() points it at the original stdout and fd 1 at stderr


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    # (--edge: the same under torch.distributed.run, whose argparse takes "--n" for an
    # ambiguous abbreviation of its own options)
    p.add_argument("--n", "--edge", dest="n", type=int, default=512, help="global grid edge (nodes)")
    p.add_argument("--path", default="auto", choices=["auto", "generic", "split", "fused"])
    p.add_argument("--reps", type=int, default=9,
                   help="repetitions of the K timed steps; value = median (BASELINE.md asks "
                        "for at least 5; more keeps the GPU busy for a visible share of the run)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=5.0,
                   help="bound on each of the two CPU baseline samples")
    p.add_argument("--rows-per-block", type=int, default=0,
                   help="fused-step y rows per block (0 = the library's automatic choice)")
    p.add_argument("--no-copy-ceiling", action="store_true",
                   help="skip the flat-copy measurement reported beside the roofline")
    p.add_argument("--no-profile", action="store_true",
                   help="no hipEvent bracketing of the launches in the timed repetitions")
    p.add_argument("--prealloc-gb", type=float, default=0.0,
                   help="measurement only: hold a device buffer of this size (torch) while the "
                        "layers are allocated (shifts their placement in HBM)")
    p.add_argument("--rccl-self", action="store_true",
                   help="one GPU: the slab is a one-rank RCCL communicator whose neighbours are "
                        "itself (gcmx_comm_init(.., 1, 0, 0, 0)): the real ncclSend/ncclRecv group "
                        "runs every step and the line carries per_rank (exchange timings)")
    p.add_argument("--no-box-state", action="store_true",
                   help="do not read / sample the GPU's amdgpu sysfs (tools/box_state.py)")
    p.add_argument("--no-clock-probe", action="store_true",
                   help="no co-resident clock-sampling wave during the timed repetitions")
    p.add_argument("--emulate-slabs", type=int, default=0, metavar="K",
                   help="one GPU: split the grid into K X-slab contexts of one in-process group "
                        "(gcmx_comm_init_local: the X-slab step schedule with its overlapped "
                        "in-step exchange, device copies instead of RCCL), one host thread each")
    return p.parse_args()


def backend():
    """(gcm_amd, gcm_amd.gcmx): the product library.  Tests only: GCM_BENCH_BACKEND
    names a module whose `gcm_amd` / `gcmx` attributes stand in for them
    (tests/bench_stub.py steps the oracle on the CPU, so the N > 1 orchestration
    -- rank spawning, the unique-id broadcast, comm_init arguments, the MAX over
    ranks, the per_rank gather -- runs under gloo without a GPU).  A line made
    through it says so in `backend` and `data`; it is never a measurement."""
    name = os.environ.get("GCM_BENCH_BACKEND")
    if name:
        mod = importlib.import_module(name)
        return mod.gcm_amd, mod.gcmx
    import gcm_amd
    from gcm_amd import gcmx
    return gcm_amd, gcmx


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(a) -> int:
    """`--gpus N` (N > 1) without a launcher: start N rank processes of this
    script, each with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT set as torch.distributed.run would, rank 0's stdout
    (the JSON line) relayed to ours, the other ranks' to stderr.  The parent
    touches no GPU (torch.cuda.device_count() does not initialise one on this
    image) and refuses to run fewer ranks than asked: too few devices is an
    error, not a one-rank run.  Returns the exit code (the first failing
    rank's; the others are then terminated)."""
    if not os.environ.get("GCM_BENCH_BACKEND"):
        import torch
        have = torch.cuda.device_count()
        if have < a.gpus:
            log(f"bench.py --gpus {a.gpus}: only {have} GPU(s) visible; refusing to run fewer ranks")
            return 2
    port = _free_port()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), GCM_BENCH_SELF_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr))
    log(f"bench.py: started {a.gpus} ranks (pids {[p.pid for p in procs]}), MASTER_PORT {port}")
    import signal
    import threading

    def forward(signum, _frame):  # a terminated job takes its ranks with it
        for p in procs:
            if p.poll() is None:
                p.terminate()
        sys.exit(128 + signum)
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    rc = 0
    while any(p.poll() is None for p in procs):  # a failed rank ends the others
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            log(f"bench.py: a rank exited with {rc}; terminating the others")
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=60)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            break
        time.sleep(0.2)
    reader.join(timeout=60)
    rc = rc or next((p.returncode for p in procs if p.returncode), 0)
    sys.stdout.write(out[0].decode() if out else "")
    sys.stdout.flush()
    return rc


def host_threads() -> int:
    """Cores this process may run on (the scheduler affinity mask)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(seconds: float):
    """Oracle (C restatement, OpenMP over x) on a bounded 3-D sample of the same
    workload (96^3 parity-random field, (4,2,1), bs 2, tau 0.9), timed at 1 thread
    and at every core the process may use (the reference CPU path is
    single-threaded; the restatement is per-node independent, so threads cannot
    change its results)."""
    from oracle import oracle as O
    N = 96
    t = O.Task(D=3, border_size=2, h=[1, 1, 1], cubics={0: ([N] * 3, [0] * 3)}, courant=0.9,
               default_material=O.Material(4, 2, 1), number_of_snaps=1)
    b = O.Engine(t).bodies[0]
    O.fill_random(b, [N, N, N], 0x5EED)

    def rate(threads):
        b.stage(0, 0.9, threads)  # warm
        steps = 0
        t0 = time.perf_counter()
        while True:
            for s in range(3):
                b.stage(s, 0.9, threads)
            steps += 1
            el = time.perf_counter() - t0
            if el >= seconds or steps >= 200:
                break
        return N ** 3 * steps / el / 1e6, steps, el

    # OpenMP threads: the CPU share the job was given (OMP_NUM_THREADS, 16 on the
    # GPU box, whose affinity mask shows all 256 cores of a shared machine), else
    # every core in the affinity mask.
    all_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or host_threads()
    r1, s1, e1 = rate(1)
    rn, sn, en = rate(all_threads)
    return {"value": rn, "unit": "Mnode-steps/s", "cores": all_threads, "kind": "port",
            "value_1thread": r1, "host_cores": os.cpu_count(),
            "sample": f"oracle C restatement (gcc -O2, no FMA), 96^3 parity-random, 3 stages "
                      f"per step: {sn} steps in {en:.1f} s on {all_threads} OpenMP threads "
                      f"(the job's CPU share; os.cpu_count() = {os.cpu_count()}, affinity "
                      f"{host_threads()}); {s1} steps in {e1:.1f} s on 1 thread"}


def copy_ceiling(ctx, step_bytes, achieved_gbps):
    """What this box's HBM gives a plain copy of the same bytes the step must
    move (half read, half written): gcmx_copy_ceiling's flat copy (double2 per
    lane, non-temporal stores; torch's copy_ measured 13 % slower), timed after
    the step's repetitions (outside them), median of 5.  The step's `achieved`
    over this rate says how close the kernel is to the memory system's practical
    limit on this box (MI355X_MICROARCH.md: ~79 % of the 8 TB/s spec for a float4
    copy; tools/copy_probe.hip measures the product layout's own copy beside a
    flat one)."""
    t = ctx.copy_ceiling_ms(int(step_bytes), 5)
    gbps = step_bytes / (t * 1e-3) / 1e9
    return {"GBps": round(gbps, 1), "frac_of_copy": round(achieved_gbps / gbps, 4),
            "how": f"gcmx_copy_ceiling: flat copy of {step_bytes / 2e9:.2f} GB (16-B loads, "
                   f"non-temporal stores, 32768x256 threads grid-stride: the fastest of the 28 shapes "
                   f"tools/copy_probe.hip times), median of 5, bytes counted read + write"}


def lib_sha256() -> str:
    """Digest of the libgcmx.so this process loaded (gcm_amd.gcmx.LIB_PATH)."""
    import hashlib
    gcmx = backend()[1]
    with open(gcmx.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_traffic(n, ranks, bucket, symbol):
    """HBM bytes per launch from profiles/pmc_traffic.json (512^3; other grids
    profiles/pmc_traffic_<n>.json: rocprofv3 FETCH_SIZE / WRITE_SIZE passes,
    tools/pmc_traffic.py), used only when that profile was
    taken of THIS library build (sha256), the same grid, rank count and kernel
    instance; otherwise (None, reason)."""
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json" if n == 512 else f"pmc_traffic_{n}.json")
    if not os.path.exists(pmc):
        return None, f"no PMC profile ({os.path.basename(pmc)})"
    try:
        rec = json.load(open(pmc))
    except Exception as e:
        return None, f"unreadable PMC profile: {e}"
    k = rec.get("kernels", {}).get(bucket)
    if not k:
        return None, f"PMC profile has no '{bucket}' kernel"
    if rec.get("n") != n or rec.get("ranks", 1) != ranks:
        return None, "PMC profile of another grid / rank count"
    if k.get("symbol") != symbol:
        return None, f"PMC profile of another kernel instance ({k.get('symbol')})"
    if rec.get("lib_sha256") != lib_sha256():
        return None, "PMC profile of another libgcmx.so build"
    return k.get("hbm_bytes_per_launch"), f"{rec.get('source')} (same build, sha256 match)"


def layer_placement(ctx) -> dict:
    """Where the two time layers live (gcmx_layer_info): device addresses and
    their residues modulo the page / fragment sizes that could matter for HBM
    channel interleaving and translation (4 KiB, 64 KiB, 2 MiB, 1 GiB)."""
    li = ctx.layer_info()
    a, b = li["a"], li["b"]
    mods = {"4K": 1 << 12, "64K": 1 << 16, "2M": 1 << 21, "1G": 1 << 30}
    return {"a": hex(a), "b": hex(b), "b_minus_a": b - a, "layer_bytes": li["layer_bytes"],
            "one_allocation": li["one_allocation"], "alloc": li.get("alloc"),
            "a_mod": {k: a % m for k, m in mods.items()},
            "b_mod": {k: b % m for k, m in mods.items()},
            "b_minus_a_mod": {k: (b - a) % m for k, m in mods.items()}}


def clock_summary(samples) -> dict:
    """Shader clock from the probe's (100 MHz ticks, cycles) samples: per
    interval Δcycles / Δticks × 100 MHz; median and 10/90 % over the intervals."""
    import numpy as np
    if len(samples) < 3:
        return {"samples": int(len(samples))}
    s = samples.astype(np.float64)
    dt = np.diff(s[:, 0])
    dc = np.diff(s[:, 1])
    ok = dt > 0
    mhz = dc[ok] / dt[ok] * 100.0
    return {"samples": int(len(samples)), "span_ms": round(float((s[-1, 0] - s[0, 0]) / 1e5), 1),
            "mhz_median": round(float(np.median(mhz)), 1),
            "mhz_p10": round(float(np.percentile(mhz, 10)), 1),
            "mhz_p90": round(float(np.percentile(mhz, 90)), 1)}


class stdout_to_stderr:
    """Sends fd 1 to fd 2 for a block: RCCL prints a version banner on stdout when
    a communicator is created, and the driver reads the ONE JSON line on stdout."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def rank_record(ctx, rank, kernels, steps_total, step_ms):
    """One rank's exchange / compute split over the timed repetitions, from the
    library's hipEvent buckets (gcmx_profile_*): the interior and boundary
    launches, the RCCL group on the comm stream from data-ready to its last
    kernel (`halo_ms`, per post), the time the compute stream stood still
    waiting for it (`exposed_wait_ms`, per step: the part of the exchange not
    hidden behind compute), the bytes one link direction carries per post and
    the rate that gives."""
    def avg(name):
        v = kernels.get(name)
        return v["total_ms"] / v["launches"] if v and v["launches"] else 0.0
    hname = "halo_rccl" if "halo_rccl" in kernels else ("halo_loopback" if "halo_loopback" in kernels else None)
    h = kernels.get(hname) if hname else None
    halo_ms = avg(hname) if hname else 0.0
    wait = kernels.get("halo_wait")
    bytes_dir = h["bytes_per_launch"] if h else 0.0
    return {"rank": rank, "step_ms": round(step_ms, 4),
            "interior_ms": round(avg("fused_xyz"), 4),
            "boundary_ms": round(avg("fused_xyz_boundary"), 4),
            "halo_ms": round(halo_ms, 4),
            "halo_posts_per_step": round(h["launches"] / steps_total, 3) if h else 0.0,
            "exposed_wait_ms": round(wait["total_ms"] / steps_total, 4) if wait else 0.0,
            "bytes_per_direction": bytes_dir,
            "GBps_per_direction": round(bytes_dir / (halo_ms * 1e-3) / 1e9, 1) if halo_ms > 0 else None,
            "transport": hname,
            "channels_per_peer": ctx.comm_channels_per_peer}


def box_summary(box, sampled):
    """The few box fields that tell ranks' GPUs apart (tools/box_state.py)."""
    import statistics
    box = box or {}
    sampled = sampled or {}
    sc = [int(k[:-3]) for k, n in (sampled.get("sclk") or {}).items() if k.endswith("Mhz") for _ in range(n)]
    return {"unique_id": box.get("unique_id"), "vbios": box.get("vbios_version"),
            "power_w": sampled.get("power_w"), "sclk_mhz_median": statistics.median(sc) if sc else None}


def multi_gpu_parity(dist, world, rank, device, U, U1, L, channels, gcm_amd):
    """N > 1 self-check of the RCCL X-slab path (halo exchange overlapped with the
    interior X stage): 3 steps on a 12*N x 40 x 64 grid split into N slabs must
    equal, bitwise, the same grid run whole on rank 0's GPU."""
    import numpy as np
    import torch
    Xs, Y, Z, bs, seed = 12, 40, 64, 2, 0x5EED
    Xg = Xs * world
    c = gcm_amd.Context(3, bs, [Xs, Y, Z], start=[rank * Xs, 0, 0], device=device)
    c.set_materials(U[None], U1[None], L[None])
    c.fill_random([Xg, Y, Z], seed)
    obj = [gcm_amd.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    # RCCL fixes the channels per peer at the process's first communicator (the
    # bench's): this one uses the same count (gcmx.h, checked contract)
    c.comm_init(obj[0], world, rank, rank - 1 if rank > 0 else -1,
                rank + 1 if rank < world - 1 else -1, global_x=Xg, channels_per_peer=channels)
    for _ in range(3):
        c.step(0.9)
    mine = c.download().reshape(Xs + 2 * bs, Y + 2 * bs, Z + 2 * bs, 9)[bs:-bs, bs:-bs, bs:-bs]
    path = c.effective_path
    c.close()
    t = torch.from_numpy(np.ascontiguousarray(mine))
    parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, parts, dst=0)
    ok = True
    if rank == 0:
        f = gcm_amd.Context(3, bs, [Xg, Y, Z], device=device)
        f.set_materials(U[None], U1[None], L[None])
        f.fill_random([Xg, Y, Z], seed)
        for _ in range(3):
            f.step(0.9)
        whole = f.download().reshape(Xg + 2 * bs, Y + 2 * bs, Z + 2 * bs, 9)[bs:-bs, bs:-bs, bs:-bs]
        f.close()
        ok = bool(np.array_equal(np.concatenate([p.numpy() for p in parts], axis=0), whole))
    res = [ok]
    dist.broadcast_object_list(res, src=0)
    return {"ok": res[0], "grid": [Xg, Y, Z], "slabs": world, "steps": 3, "path": path}


def emulate_slabs(a):
    """--emulate-slabs K on one GPU: the config-3 decomposition (K X slabs of the
    N^3 grid) as the ranks of an in-process group, so every step runs the exact
    code RCCL ranks run -- interior beside the boundary planes, the new boundary
    planes posted while the interior runs, the next step's boundary waiting for
    them -- with device copies for the exchange.  All K slabs share the one GPU,
    so the group's step time is the sum of K ranks' work plus the copies; the
    per-rank figure divides it by K (the chip is work-conserving across the
    slabs' streams).  Compared with one undivided context on the same GPU."""
    import gcm_amd
    from gcm_amd import gcmx
    from gcm_amd.host import isotropic_elastic_matrices
    N, K = a.n, a.emulate_slabs
    if N % K:
        raise SystemExit("grid edge must be divisible by the number of slabs")
    X = N // K
    U, U1, L = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
    tau = 0.9
    slabs = []
    for r in range(K):
        c = gcm_amd.Context(3, 2, [X, N, N], start=[r * X, 0, 0], device=0)
        c.set_materials(U[None], U1[None], L[None])
        c.fill_random([N, N, N], 0x5EED)
        slabs.append(c)
    gcmx.comm_init_local(slabs)
    gcmx.local_group_steps(slabs, tau, max(1, a.warmup))
    for c in slabs:
        c.profile(True)
        c.profile_reset()
    rep_s = []
    for _ in range(max(1, a.reps)):
        t0 = time.perf_counter()
        gcmx.local_group_steps(slabs, tau, a.steps)  # ends with every slab synced
        rep_s.append(time.perf_counter() - t0)
    kern = {}
    for c in slabs:
        for k, v in c.profile_read().items():
            d = kern.setdefault(k, {"total_ms": 0.0, "launches": 0, "kernel": v["kernel"]})
            d["total_ms"] += v["total_ms"]
            d["launches"] += v["launches"]
    paths = sorted({c.last_path for c in slabs})
    for c in slabs:
        c.close()
    el = sorted(rep_s)[len(rep_s) // 2]
    # the same grid as one context, same GPU, same repetitions
    w = gcm_amd.Context(3, 2, [N, N, N], device=0)
    w.set_materials(U[None], U1[None], L[None])
    w.fill_random([N, N, N], 0x5EED)
    for _ in range(max(1, a.warmup)):
        w.step(tau)
    w.sync()
    whole = []
    for _ in range(max(1, a.reps)):
        w.sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            w.step(tau)
        w.sync()
        whole.append(time.perf_counter() - t0)
    w.close()
    ew = sorted(whole)[len(whole) // 2]
    ms = el / a.steps * 1e3
    msw = ew / a.steps * 1e3
    out = {
        "metric": "Mnode-steps/sec, 3D isotropic elastic CubicGrid, X-slab group emulated on one GPU",
        "value": round(N ** 3 * a.steps / el / 1e6, 1), "unit": "Mnode-steps/s", "n_gpus": 1,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4),
        "rep_ms_per_step": [round(r / a.steps * 1e3, 4) for r in rep_s],
        "higher_is_better": True, "dtype": "f64", "data": "synthetic parity-random field (seed 0x5EED)",
        "config": {"workload": f"3-D isotropic elastic CubicGrid {N}^3 as {K} X slabs of {X} x {N} x {N}, "
                               f"borderSize 2, tau 0.9", "slabs": K, "paths": paths,
                   "parallelism": f"x-slab{K} in-process group on one GPU (gcmx_comm_init_local, "
                                  f"one host thread per slab, device-copy exchange)"},
        "per_rank_ms_per_step": round(ms / K, 4),
        "whole_grid_ms_per_step": round(msw, 4),
        "decomposition_overhead": round(ms / msw, 4),
        # K ranks contending for ONE GPU (their boundary launches, interiors and
        # copies interleaved on one chip): a pessimistic stand-in for K GPUs.  One
        # rank's own step with the exchange in flight is scripts/bench_slab.py
        # --loop-gbps (loopback transport), DESIGN.md §5.
        "speedup_if_ranks_ran_this_fast_on_K_gpus": round(K * msw / ms, 3),
        "note": "all K ranks share one GPU; per-rank step with the exchange in flight: "
                "scripts/bench_slab.py --loop-gbps (DESIGN.md §5)",
        "kernels": {k: {"avg_ms": round(v["total_ms"] / max(1, v["launches"]), 4),
                        "launches_per_step": round(v["launches"] / (a.steps * max(1, a.reps)), 2),
                        "kernel": v["kernel"]} for k, v in kern.items()},
    }
    print(json.dumps(out), file=JSON_OUT, flush=True)


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and not a.emulate_slabs:
        sys.exit(self_launch(a))
    # The ONE JSON line goes to the original stdout; everything else the
    # libraries write to fd 1 (RCCL prints a version banner when a communicator
    # is created) goes to stderr.
    global JSON_OUT
    sys.stdout.flush()
    JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if a.emulate_slabs:
        return emulate_slabs(a)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE (the launcher's rank count)")
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    gcm_amd, gcmx = backend()
    stub = os.environ.get("GCM_BENCH_BACKEND")
    paths = {"auto": gcmx.PATH_AUTO, "generic": gcmx.PATH_GENERIC, "split": gcmx.PATH_SPLIT,
             "fused": gcmx.PATH_FUSED}

    N = a.n
    if N % world:
        raise SystemExit("grid edge must be divisible by the number of ranks")
    X = N // world
    x0 = rank * X
    device = local if torch.cuda.device_count() > 1 else 0
    # material (4,2,1): ElasticModel<3> matrices built by the host mirror
    from gcm_amd.host import isotropic_elastic_matrices  # host C++ (ElasticModel), no GPU
    U, U1, L = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)
    tau = 0.9 * 1.0 / 1.0  # Courant * h / max|lambda| (Engine.cpp:124-140)

    box = None
    if not a.no_box_state:  # every rank reads its own GPU's state (per_rank for N > 1)
        try:
            box = box_state.static_state(device)
        except Exception as e:  # reported context, never required
            box = {"error": str(e)}
    t_setup = time.perf_counter()
    hold = None
    if a.prealloc_gb > 0:  # measurement only: shifts the layers' placement
        hold = torch.empty(int(a.prealloc_gb * (1 << 30)), dtype=torch.uint8, device=f"cuda:{device}")
    ctx = gcm_amd.Context(3, 2, [X, N, N], start=[x0, 0, 0], device=device)
    placement = layer_placement(ctx)
    ctx.set_materials(U[None], U1[None], L[None])
    ctx.set_path(paths[a.path])
    if a.rows_per_block:
        ctx.set_schedule(gcmx.SCHED_AUTO, a.rows_per_block)
    ctx.fill_random([N, N, N], 0x5EED)
    ctx_fp = ctx.fp_mode
    if world > 1:
        uid = gcm_amd.unique_id() if rank == 0 else None
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        ctx.comm_init(obj[0], world, rank, rank - 1 if rank > 0 else -1,
                      rank + 1 if rank < world - 1 else -1, global_x=N)
    elif a.rccl_self:
        ctx.comm_init(gcm_amd.unique_id(), 1, 0, 0, 0)
    ctx.sync()
    parity = None
    if world > 1:
        parity = multi_gpu_parity(dist, world, rank, device, U, U1, L, ctx.comm_channels_per_peer, gcm_amd)
        log(f"[rank {rank}] multi-GPU slab parity: {parity}")
    log(f"[rank {rank}] slab x[{x0},{x0 + X}) of {N}^3, {ctx.device_bytes / 1e9:.1f} GB, "
        f"path {ctx.effective_path}, setup {time.perf_counter() - t_setup:.1f}s")

    def barrier():
        if dist is not None:
            dist.barrier()

    tw = time.perf_counter()
    for _ in range(a.warmup):
        ctx.step(tau)
    ctx.sync()
    warm_ms = (time.perf_counter() - tw) / max(1, a.warmup) * 1e3
    # one co-resident wave samples the shader clock over the timed repetitions
    clock = None
    if not a.no_clock_probe:
        span = min(20.0, max(0.2, 1.15 * a.reps * a.steps * warm_ms * 1e-3 + 0.05))
        ctx.clock_probe_start(span, max(50.0, span * 1e6 / 4000))

    # K timed steps, repeated `reps` times (median reported).  When profiling,
    # every launch in these same repetitions is bracketed by hipEvents on the
    # stream it runs on (gcmx_profile_enable), which is where kernel_avg_ms
    # comes from.
    if not a.no_profile:
        ctx.profile(True)
        ctx.profile_reset()
    sampler = None
    if not a.no_box_state:
        try:
            sampler = box_state.Sampler(device).start()
        except Exception as e:  # reported context, never required
            log(f"box-state sampler failed: {e}")
    rep_s = []
    rep_kernels = []  # per repetition: the profile's totals accumulated in that repetition
    prev = {}
    for _ in range(max(1, a.reps)):
        barrier()
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ctx.step(tau)
        ctx.sync()
        barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            tt = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        rep_s.append(el)
        if not a.no_profile:
            cur = ctx.profile_read()
            rep_kernels.append({k: (v["total_ms"] - prev.get(k, {}).get("total_ms", 0.0),
                                    v["launches"] - prev.get(k, {}).get("launches", 0))
                                for k, v in cur.items()})
            prev = cur
    sampled = sampler.stop() if sampler is not None else None
    if not a.no_clock_probe:
        clock = clock_summary(ctx.clock_probe_read())
    kernels = {}
    if not a.no_profile:
        kernels = ctx.profile_read()
        ctx.profile(False)
    el = sorted(rep_s)[len(rep_s) // 2]
    per_rank = None
    if (world > 1 or a.rccl_self) and kernels:
        rec = rank_record(ctx, rank, kernels, a.steps * max(1, a.reps), el / a.steps * 1e3)
        rec["box"] = box_summary(box, sampled)
        if dist is not None:
            recs = [None] * world if rank == 0 else None
            dist.gather_object(rec, recs, dst=0)
            per_rank = recs
        else:
            per_rank = [rec]
    # the kernel statistic that matches ms_per_step: the median over the
    # repetitions of each repetition's mean launch duration
    rep_avg = {}
    for k in kernels:
        avgs = sorted(t / n for t, n in (r.get(k, (0.0, 0)) for r in rep_kernels) if n > 0)
        if avgs:
            rep_avg[k] = avgs[len(avgs) // 2]

    total_nodes = N ** 3
    value = total_nodes * a.steps / el / 1e6
    roof = None
    if kernels:
        # the dominant COMPUTE kernel (the exchange buckets time the comm stream
        # and the compute stream's waits, not a kernel of the step)
        comp = {k: v for k, v in kernels.items() if not k.startswith("halo_")} or kernels
        dom_name, dom = max(comp.items(), key=lambda kv: kv[1]["total_ms"])
        mean_ms = dom["total_ms"] / max(1, dom["launches"])
        avg_ms = rep_avg.get(dom_name, mean_ms)
        achieved = dom["bytes_per_launch"] / (avg_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(N, world, dom_name, dom["kernel"])
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": dom_name,
                # median over the repetitions of each one's mean launch time (the same
                # statistic as ms_per_step); the mean over every launch beside it
                "kernel_avg_ms": round(avg_ms, 4), "kernel_mean_all_ms": round(mean_ms, 4),
                # the instance the library reports it launched (gcmx_profile_kernel)
                "kernel_symbol": dom["kernel"],
                "algorithmic_bytes_per_launch": dom["bytes_per_launch"],
                "kernels": {k: {"avg_ms": round(v["total_ms"] / max(1, v["launches"]), 4),
                                "GBps": round(v["bytes_per_launch"] /
                                              (v["total_ms"] / max(1, v["launches"]) * 1e-3) /
                                              1e9, 1) if v["total_ms"] > 0 else None}
                            for k, v in kernels.items()}}

    if roof is not None and not a.no_copy_ceiling:
        try:
            roof["copy_ceiling"] = copy_ceiling(ctx, dom["bytes_per_launch"], roof["achieved"])
        except Exception as e:  # reported context, never required
            log(f"copy ceiling failed: {e}")

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            cpu = cpu_baseline(a.cpu_seconds)
        except Exception as e:  # the baseline is reported, never required
            log(f"cpu baseline failed: {e}")

    if rank == 0:
        step_bytes = 3 * BYTES_PER_NODE_STAGE * total_nodes  # three separate stage passes
        out = {
            # BASELINE.json's metric when N = 512; other grids name their own size
            "metric": f"Mnode-steps/sec + achieved HBM GB/s, 3D isotropic elastic {N}³ CubicGrid",
            "value": round(value, 1),
            "unit": "Mnode-steps/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 4),
            "reps": len(rep_s),
            "rep_ms_per_step": [round(r / a.steps * 1e3, 4) for r in rep_s],
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("STUB BACKEND (tests only, not a measurement): " if stub else "")
                    + "synthetic parity-random field (SplitMix64 seed 0x5EED), material (4,2,1)",
            **({"backend": f"{stub} (test stub)"} if stub else {}),
            "config": {"workload": f"3-D isotropic elastic CubicGrid {N}^3, borderSize 2, "
                                   f"Courant 0.9, tau 0.9, one full time step (3 stages)",
                       "global_nodes": total_nodes, "slabs": world, "path": ctx.effective_path,
                       # who started the ranks: bench.py itself (--gpus N, no launcher), a
                       # launcher (torch.distributed.run), or one process
                       "launch": ("bench.py self-launch" if os.environ.get("GCM_BENCH_SELF_LAUNCHED")
                                  else "launcher" if "WORLD_SIZE" in os.environ else "single process"),
                       "parallelism": f"x-slab{world}" if world > 1 else
                                      ("single, RCCL self-exchange (one-rank communicator)" if a.rccl_self else "single"),
                       **({"rccl_channels_per_peer": ctx.comm_channels_per_peer} if world > 1 or a.rccl_self else {}),
                       # the one-pass step's floating-point build (gcmx_set_fp_mode): "fma" =
                       # multiply-adds contracted, the product default, held to the north
                       # star's 1e-10 relative L2 of the reference (tests/test_gpu_fma.py);
                       # "exact" = the reference's roundings, bitwise (GCMX_FP=exact)
                       "fp": "exact" if ctx_fp == gcmx.FP_EXACT else "fma",
                       **({"rows_per_block": a.rows_per_block} if a.rows_per_block else {})},
            # NOT an HBM rate: the bytes three separate stage passes (SURVEY §8d, 432 B per
            # node-step) would move, over the measured step time; the one-pass step moves 144 B
            "equivalent_GBps_if_three_stage_passes": round(step_bytes * a.steps / el / 1e9, 1),
            "roofline": roof,
            "cpu_baseline": cpu,
            "multi_gpu_parity": parity,
            # N > 1 (or --rccl-self): every rank's exchange / compute split (rank_record)
            "per_rank": per_rank,
            # what distinguishes one process's run from another's on the same box
            # (VERDICT r3 item 1): the layers' placement, the clock under load,
            # the allocation order
            "process_state": {"layers": placement, "clock": clock,
                              # the box: partition modes, power cap,
                              # firmware, DPM tables (tools/box_state.py), and the DPM
                              # levels / power / temperatures sampled during the reps
                              "box": box, "box_during_reps": sampled,
                              "alloc_order": (f"torch buffer {a.prealloc_gb} GiB, " if hold is not None else "")
                                             + (f"layers A+gap+B in one block ({placement['alloc']})"
                                                if placement["one_allocation"] else "layer A, layer B, tables"),
                              "env": {k: os.environ[k] for k in ("GCMX_LAYER_GAP", "GCMX_STREAM_PRIO", "GCMX_FP", "GCMX_ALLOC")
                                      if k in os.environ},
                              "under_profiler": bool(os.environ.get("ROCPROF_OUTPUT_PATH") or
                                                     "rocprof" in os.environ.get("LD_PRELOAD", ""))},
        }
        print(json.dumps(out), file=JSON_OUT, flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
