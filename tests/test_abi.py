"""The C-ABI library loads on a CPU-only host and exports every entry point
include/gcmx.h declares (no compute calls: no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "gcmx.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b((?:gcmx|gsx)_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("gcmx_create", "gcmx_stage", "gcmx_step", "gcmx_set_materials", "gcmx_upload",
              "gcmx_download", "gcmx_halo_exchange", "gcmx_border_fill", "gcmx_copy_box"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    import gcm_amd
    lib = gcm_amd.lib()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    from gcm_amd.gcmx import SYMBOLS
    assert sorted(SYMBOLS) == declared_symbols()


def test_channels_rule_is_rank_consistent():
    """the automatic RCCL channels-per-peer rule
    (gcmx_comm_channels_rule, a pure function: no GPU call with an explicit CU
    count) must give every rank of one grid the same count -- both ends of a
    p2p connection use it -- however ragged the split: each rank calls it with
    its OWN slab width, and the multi-rank form depends only on the shared
    global X extent (the thinnest slab of an even split)."""
    from gcm_amd import gcmx
    splits = [([9, 6, 7], 40, 64), ([7, 5, 9, 3], 40, 64), ([5, 8, 3], 24, 64),
              ([256, 256], 512, 512), ([128] * 4, 512, 512), ([64] * 8, 512, 512),
              ([60, 68, 64, 64, 64, 64, 64, 64], 512, 512)]
    for xs, Y, Z in splits:
        gx, n = sum(xs), len(xs)
        vals = {gcmx.channels_rule(gx, n, x, Y, Z) for x in xs}
        assert len(vals) == 1, (xs, vals)
        # = the one-rank rule on the thinnest slab of an even split
        assert vals == {gcmx.channels_rule(0, 1, gx // n, Y, Z)}, (xs, vals)
    # 512^3 on 256 CUs: 64-plane slabs leave 16 CUs beside the
    # interior (4 channels), 128-plane slabs 8 (2), 256-plane slabs 4 (RCCL's default)
    assert gcmx.channels_rule(512, 8, 64, 512, 512) == 4
    assert gcmx.channels_rule(512, 4, 128, 512, 512) == 2
    assert gcmx.channels_rule(512, 2, 256, 512, 512) == 0
    # without the global extent a multi-rank rule cannot be rank-consistent: RCCL's default
    assert gcmx.channels_rule(0, 3, 9, 40, 64) == 0
    assert gcmx.channels_rule(512, 0, 64, 512, 512) == -1  # invalid


def test_cpu_only_calls_fail_loudly():
    """No silent fallback: without a GPU, creating a context is an error."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present")
    import gcm_amd
    assert gcm_amd.lib().gcmx_abi_version() == 3
    assert gcm_amd.lib().gcmx_pde_size(3) == 9
    with pytest.raises(gcm_amd.GcmxError):
        gcm_amd.Context(3, 2, [8, 8, 8])


def test_host_matrices_match_oracle_bitwise():
    import numpy as np
    from gcm_amd.host import isotropic_elastic_matrices as P
    from oracle.oracle import isotropic_elastic_matrices as O
    rng = np.random.default_rng(1)
    for D in (1, 2, 3):
        for _ in range(200):
            m = (rng.uniform(0.01, 100), rng.uniform(0, 1e6), rng.uniform(1, 1e6))
            for x, y in zip(P(D, *m), O(D, *m)):
                assert np.array_equal(x, y)
                assert np.array_equal(np.signbit(x), np.signbit(y))
