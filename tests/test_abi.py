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
