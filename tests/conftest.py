import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# The suite compares the GPU with the oracle BITWISE, i.e. in the exact build of
# the one-pass step (gcmx_set_fp_mode GCMX_FP_EXACT); every context a test
# creates starts in it.  The product default (GCMX_FP_FMA, multiply-adds
# contracted) is tested against the north-star tolerance in test_gpu_fma.py,
# which sets the mode per context.
os.environ["GCMX_FP"] = "exact"
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle as O
    O.build()
    return O


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gcmx():
    """The product library; on a GPU box it must load (no fallback)."""
    import gcm_amd
    gcm_amd.lib()
    return gcm_amd
