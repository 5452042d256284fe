"""bench.py's N > 1 orchestration on the CPU (gloo), with the product library
replaced by tests/bench_stub.py (oracle stages + a gloo X-slab exchange).

What runs is bench.py's own code: the ranks it starts itself when no launcher
set WORLD_SIZE (or torch.distributed.run's), the unique-id broadcast, the
comm_init arguments (neighbours, global_x), the MAX of the repetition times
over ranks, the per_rank gather and multi_gpu_parity's slab concatenation
against a whole-grid run (the reference's X-slab test, src/test/TestMPI.cpp:92-155,
ASSERT_EQ at :150)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--gpus", "2", "--edge", "16", "--steps", "2", "--warmup", "1", "--reps", "3", "--no-box-state",
        "--no-clock-probe", "--no-copy-ceiling"]


def _env(tmp_path, **extra):
    env = dict(os.environ, GCM_BENCH_BACKEND="tests.bench_stub", GCM_BENCH_STUB_LOG=str(tmp_path),
               PYTHONPATH=ROOT, **extra)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _run(cmd, env):
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, f"expected ONE JSON line on stdout, got {len(lines)}: {p.stdout[-2000:]}"
    return json.loads(lines[0])


def _check(d, tmp_path, world=2, n=16):
    assert d["n_gpus"] == world
    assert d["backend"].startswith("tests.bench_stub") and d["data"].startswith("STUB")
    assert d["config"]["slabs"] == world and d["config"]["parallelism"] == f"x-slab{world}"
    assert d["metric"].endswith(f"{n}³ CubicGrid")
    # multi_gpu_parity: the N slabs concatenated == the grid run whole on rank 0
    par = d["multi_gpu_parity"]
    assert par["ok"] is True and par["slabs"] == world and par["grid"] == [12 * world, 40, 64]
    # per_rank: one record per rank, gathered on rank 0; their step times are the
    # all_reduce MAX (identical on every rank, and the line's ms_per_step)
    pr = d["per_rank"]
    assert [r["rank"] for r in pr] == list(range(world))
    assert len({r["step_ms"] for r in pr}) == 1 and pr[0]["step_ms"] == d["ms_per_step"]
    assert all(r["transport"] == "halo_rccl" and r["halo_posts_per_step"] == 1.0 for r in pr)
    assert len(d["rep_ms_per_step"]) == 3
    logs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    # distinct processes, one per rank
    assert len({l["pid"] for l in logs}) == world and [l["rank"] for l in logs] == list(range(world))
    # rank 0 made the unique ids (the bench communicator, then multi_gpu_parity's);
    # every rank initialised its communicators with exactly those, in that order
    uids = logs[0]["unique_ids"]
    assert len(uids) == 2 and all(not l["unique_ids"] for l in logs[1:])
    X = n // world
    for r, l in enumerate(logs):
        ci = l["comm_init"]
        assert [c["uid"] for c in ci] == uids
        for c, gx, xs in ((ci[0], n, X), (ci[1], 12 * world, 12)):
            assert c["nranks"] == world and c["rank"] == r
            assert c["left"] == (r - 1 if r > 0 else -1) and c["right"] == (r + 1 if r < world - 1 else -1)
            assert c["global_x"] == gx and c["sizes"][0] == xs and c["start"][0] == r * xs
        # the parity communicator takes the bench communicator's channel count
        assert ci[1]["channels_per_peer"] == 4
        # one exchange per step of both communicators: warmup + reps * steps, + 3
        assert l["exchanges"] == 1 + 3 * 2 + 3


def test_bench_starts_its_own_ranks_without_a_launcher(tmp_path):
    """`python bench.py --gpus 2` with no WORLD_SIZE: bench.py starts the two
    ranks itself (no silent one-rank run)."""
    d = _run([sys.executable, "bench.py"] + ARGS, _env(tmp_path))
    _check(d, tmp_path)
    assert d["config"]["launch"] == "bench.py self-launch"


def test_bench_under_torch_distributed_run(tmp_path):
    """The driver's form: torch.distributed.run sets the rank variables."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py"] + ARGS, _env(tmp_path))
    _check(d, tmp_path)
    assert d["config"]["launch"] == "launcher"


def test_bench_parity_check_sees_a_missing_exchange(tmp_path):
    """multi_gpu_parity is a real check: with the stub's exchange switched off
    the slabs differ from the whole grid and the line says so."""
    d = _run([sys.executable, "bench.py"] + ARGS, _env(tmp_path, GCM_BENCH_STUB_NO_EXCHANGE="1"))
    assert d["multi_gpu_parity"]["ok"] is False


def test_bench_refuses_more_gpus_than_visible(tmp_path):
    """No stub, no GPU here: --gpus 2 must fail, not measure one rank."""
    env = _env(tmp_path)
    env.pop("GCM_BENCH_BACKEND")
    p = subprocess.run([sys.executable, "bench.py"] + ARGS, cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode != 0 and not p.stdout.strip()
    assert "refusing to run fewer ranks" in p.stderr


def test_bench_rank_failure_ends_the_job(tmp_path):
    """A rank that dies takes the self-launched job down with a non-zero exit
    (the other rank is terminated, not left waiting in a collective)."""
    env = _env(tmp_path, GCM_BENCH_STUB_FAIL_RANK="1")
    p = subprocess.run([sys.executable, "bench.py"] + ARGS, cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode != 0 and not p.stdout.strip()
