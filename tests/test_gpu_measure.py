"""Measurement helpers of the C-ABI on the GPU (bench.py's roofline fields)."""
import pytest

pytestmark = pytest.mark.gpu


def test_copy_ceiling_reports_a_plausible_rate():
    """gcmx_copy_ceiling: a flat 256 MB copy runs between 0.5 and 8 TB/s (the HBM
    spec), and bad arguments are refused."""
    import gcm_amd
    from gcm_amd.gcmx import GcmxError
    c = gcm_amd.Context(3, 2, [8, 8, 8])
    try:
        nbytes = 256 << 20
        ms = c.copy_ceiling_ms(nbytes, 3)
        gbps = nbytes / (ms * 1e-3) / 1e9
        assert 500.0 < gbps < 8000.0, gbps
        with pytest.raises(GcmxError):
            c.copy_ceiling_ms(nbytes, 0)
    finally:
        c.close()


@pytest.mark.timeout(240)
def test_bench_prints_one_json_line_with_rccl_self():
    """The driver reads ONE JSON line from bench.py's stdout.  With an RCCL
    communicator in the process (RCCL prints a version banner on stdout when one
    is created) the line must still be the only stdout output, and an exchange
    run carries per_rank with the exchange timings and the rank's box summary."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--n", "64", "--steps", "3",
                        "--warmup", "1", "--reps", "2", "--rccl-self", "--no-cpu-baseline",
                        "--no-copy-ceiling", "--no-clock-probe"],
                       capture_output=True, text=True, timeout=200, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["roofline"]["kernel"] == "fused_xyz"
    pr = d["per_rank"]
    assert len(pr) == 1 and pr[0]["halo_ms"] > 0 and pr[0]["transport"] == "halo_rccl"
    assert pr[0]["halo_posts_per_step"] == 1.0 and pr[0]["bytes_per_direction"] > 0
    assert "box" in pr[0] and "process_state" in d


@pytest.mark.timeout(120)
def test_bench_refuses_more_ranks_than_gpus():
    """`bench.py --gpus N` without a launcher starts N ranks itself -- and on a
    box with fewer than N GPUs it must fail before touching one, not measure a
    single rank.  N = the visible GPUs + 1, so no rank starts."""
    import os
    import subprocess
    import sys
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n), "--n", "64", "--steps", "1"],
                       capture_output=True, text=True, timeout=100, cwd=root, env=env)
    assert r.returncode != 0 and not r.stdout.strip()
    assert "refusing to run fewer ranks" in r.stderr
