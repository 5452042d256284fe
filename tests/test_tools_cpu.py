"""CPU tests of the measurement helpers: the PMC record's kernel naming
(tools/pmc_traffic.py) must match the symbols the library reports
(gcmx_profile_kernel), and bench.py uses a PMC record only for the build, grid
and instance it was taken of."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import pmc_traffic  # noqa: E402


def test_readable_matches_the_library_symbols():
    r = pmc_traffic.readable
    assert r("void gcmx::xyz_fma::k_step_tx2<2, 512, true, true, false, false, false>(double const*)") == \
        "k_step_tx2<2, 512, KF0, UNI, !FACES, FMA>"
    assert r("void gcmx::xyz_exact::k_step_tx2<2, 256, true, false, true, false, false>(x)") == \
        "k_step_tx2<2, 256, KF0, !UNI, FACES>"
    assert r("void gcmx::xyz_fma::k_step_tx2<2, 512, true, true, false, false, true>(x)") == \
        "k_step_tx2<2, 512, KF0, UNI, !FACES, ZS, FMA>"
    assert r("void gcmx::xyz_fma::k_step_tx2<2, 64, true, true, true, true, false>(x)") == \
        "k_step_tx2<2, 64, KF0, UNI, FACES, HET, FMA>"
    assert r("void gcmx::xyz_fma::k_fused_xyz<3, 1024, true, true>(x)") == "k_fused_xyz<3, 1024, KF0, UNI, FMA>"


def test_the_committed_pmc_records_name_their_grid_and_instance():
    for n, name, sym in ((512, "pmc_traffic.json", "k_step_tx2<2, 512, KF0, UNI, !FACES, FMA>"),
                         (256, "pmc_traffic_256.json", "k_step_tx2<2, 256, KF0, UNI, !FACES, FMA>"),
                         (1024, "pmc_traffic_1024.json", "k_step_tx2<2, 512, KF0, UNI, !FACES, ZS, FMA>")):
        rec = json.load(open(os.path.join(ROOT, "profiles", name)))
        k = rec["kernels"]["fused_xyz"]
        assert rec["n"] == n and rec["ranks"] == 1 and k["symbol"] == sym
        # corrected PMC bytes: at least the compulsory read + write, at most 1.3x
        assert 1.0 <= k["traffic_over_algorithmic"] < 1.3
        assert k["algorithmic_bytes_per_launch"] == 144 * n ** 3


def test_bench_uses_a_pmc_record_only_when_everything_matches(monkeypatch):
    rec = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    sym = rec["kernels"]["fused_xyz"]["symbol"]
    monkeypatch.setattr(bench, "lib_sha256", lambda: rec["lib_sha256"])
    t, why = bench.pmc_traffic(512, 1, "fused_xyz", sym)
    assert t == rec["kernels"]["fused_xyz"]["hbm_bytes_per_launch"] and "sha256 match" in why
    assert bench.pmc_traffic(512, 8, "fused_xyz", sym)[0] is None           # other rank count
    assert bench.pmc_traffic(512, 1, "fused_xyz", sym + "x")[0] is None     # other instance
    assert bench.pmc_traffic(128, 1, "fused_xyz", sym)[0] is None           # no record for the grid
    monkeypatch.setattr(bench, "lib_sha256", lambda: "0" * 64)
    t, why = bench.pmc_traffic(512, 1, "fused_xyz", sym)
    assert t is None and "another libgcmx.so build" in why


def test_rank_record_from_profile_buckets():
    """bench.rank_record turns the library's hipEvent buckets into one rank's
    exchange / compute split (per post and per step)."""
    class C:
        comm_channels_per_peer = 4
    k = {"fused_xyz": {"total_ms": 47.0, "launches": 100, "kernel": "k", "bytes_per_launch": 1.0},
         "fused_xyz_boundary": {"total_ms": 7.0, "launches": 100, "kernel": "k", "bytes_per_launch": 1.0},
         "halo_rccl": {"total_ms": 44.0, "launches": 100, "kernel": "rccl", "bytes_per_launch": 26947584.0},
         "halo_wait": {"total_ms": 1.0, "launches": 100, "kernel": "wait", "bytes_per_launch": 0.0}}
    r = bench.rank_record(C(), 3, k, 100, 0.56)
    assert r["rank"] == 3 and r["interior_ms"] == 0.47 and r["boundary_ms"] == 0.07
    assert r["halo_ms"] == 0.44 and r["halo_posts_per_step"] == 1.0 and r["exposed_wait_ms"] == 0.01
    assert r["GBps_per_direction"] == round(26947584.0 / 0.44e-3 / 1e9, 1) and r["transport"] == "halo_rccl"
