"""Layout independence: the suites' cases re-run with the
device strides no longer implied by the grid sizes.

GCMX_ROW_PAD / GCMX_PLANE_PAD / GCMX_CS_PAD (read by gcmx_create, tests only)
pad every row, every 3-D x plane and every component plane.  Each kernel, the
host conversions (upload / download / fill_random / material ids) and the C++
engine must take every offset from the library's Geo, so every case below must
pass unchanged -- bitwise where the original asserts bitwise.  A round-5 tuning
build with such padding failed the C++ engine's two-layer case
(test_fma_engine_two_layers[rho], relative L2 0.377); these cases keep that
class of fault from shipping.  The test functions are the other modules' own,
collected again here under the autouse padding fixture."""
import pytest

from tests.test_gpu_2d import test_step2d_faces_matches_oracle, test_step2d_matches_oracle  # noqa: F401
from tests.test_gpu_engine import (test_engine_adhesion_contact, test_engine_anchor_3d,  # noqa: F401
                                   test_engine_maxwell_ode, test_engine_stack_two_materials_and_maxwell,
                                   test_engine_two_layers)
from tests.test_gpu_faces import (test_engine_partial_faces_one_pass, test_step_face_map_matches_oracle,  # noqa: F401
                                  test_step_faces_heterogeneous_one_pass, test_step_faces_matches_oracle)
from tests.test_gpu_fma import (test_fma_engine_two_layers, test_fma_engine_xbodies_equal_one_body,  # noqa: F401
                                test_fma_heterogeneous_within_tolerance, test_fma_step_within_tolerance)
from tests.test_gpu_parity import (test_adhesion_contact_two_contexts_bitwise, test_border_fill_matches_oracle,  # noqa: F401
                                   test_fused_step_3d, test_generic_stages_random_with_ghosts,
                                   test_heterogeneous_materials, test_heterogeneous_one_pass_step_matches_oracle,
                                   test_heterogeneous_step_ode_fused_equals_step_then_ode, test_split_stages_3d,
                                   test_x_slabs_with_copy_halo_equal_single, test_zsplit_step_matches_oracle)
from tests.test_gpu_slabs import test_local_group_fused_equals_whole, test_rccl_self_exchange  # noqa: F401

pytestmark = pytest.mark.gpu

PADS = {"GCMX_ROW_PAD": "16", "GCMX_PLANE_PAD": "64", "GCMX_CS_PAD": "512"}


@pytest.fixture(autouse=True)
def padded_layout(monkeypatch):
    for k, v in PADS.items():
        monkeypatch.setenv(k, v)
    yield


@pytest.fixture(scope="module")
def G():
    import gcm_amd
    gcm_amd.lib()
    return gcm_amd


@pytest.fixture(scope="module")
def H():
    from gcm_amd import _gcm_host
    return _gcm_host


def test_padding_reaches_the_geometry(G):
    """The knobs are in effect: the strides are the padded ones."""
    import os
    c = G.Context(3, 2, [6, 20, 64], device=0)
    g = c.geometry()
    c.close()
    row = 96 + int(os.environ["GCMX_ROW_PAD"])  # 14 lead + 2 + 64 + 2 -> 96 (16-aligned), + pad
    assert g["stride"][1] == row
    assert g["stride"][0] == row * 24 + int(os.environ["GCMX_PLANE_PAD"])
    assert g["cs"] >= g["stride"][0] * 10 + int(os.environ["GCMX_CS_PAD"])
