"""GPU-free half of the C++ host mirror: HipMesh::setUpPde's host state
(MaterialsCondition::apply + InitialCondition::apply, DefaultMesh.hpp:60-66)
built by gcm_amd._gcm_host.host_state must equal, bitwise, the oracle Body's
set-up for the same Task -- every area kind, vectors, waves, quantities, body
materials, 1-D/2-D/3-D, offset starts and anisotropic h."""
import numpy as np
import pytest

from oracle import oracle as O
from tests.taskspec import host_task, oracle_task, spec


@pytest.fixture(scope="module")
def H():
    from gcm_amd import _gcm_host
    return _gcm_host


CASES = {
    "sphere_pressure_3d": spec(3, 2, [1, 1, 1], {0: ([16] * 3, [0] * 3)}, 0.9, (4, 2, 1), snaps=1,
                               quantities=[(("sphere", 4, (8, 8, 8)), "PRESSURE", 10.0)]),
    "wave_1d": spec(1, 2, [1], {0: ([300], [0])}, 0.9, (4, 2, 1), snaps=1,
                    waves=[(("box", (100, -1, -1), (200, 1, 1)), "P_FORWARD", 0, "Vx", 1.0)]),
    "run_statement_2d": spec(2, 5, [7.0 / 19, 3.0 / 39], {0: ([20, 40], [0, 0])}, 4.5,
                             (4, 2, 0.5), snaps=9,
                             waves=[(("box", (-1, 0.1125, -1), (8, 0.6375, 1)), "S1_FORWARD", 1,
                                     "Vx", 1.0)]),
    "two_layers_2d": spec(2, 3, [2.0 / 49, 1.0 / 99], {0: ([50, 100], [0, 0])}, 1.5, (1, 2, 0.8),
                          inhomogeneities=[(("box", (-10, 0.5 - 1e-5, -10), (10, 10, 10)),
                                            (4, 2, 0.8))], snaps=1,
                          waves=[(("box", (-1, 0.015, -1), (4, 0.455, 1)), "P_FORWARD", 1, "Vy",
                                  -2.0)]),
    "areas_3d": spec(3, 2, [0.5, 1.0, 0.75], {0: ([14, 11, 16], [2, 0, 1])}, 0.7, (4, 2, 1),
                     inhomogeneities=[(("sphere", 2.5, (4, 5, 6)), (2, 1, 1.5)),
                                      (("cylinder", 1.5, (0, 0, 0), (8, 11, 12)), (3, 0.5, 2))],
                     snaps=4,
                     vectors=[(("box", (1, 1, 1), (6, 8, 9)), [0.1 * i for i in range(9)])],
                     waves=[(("box", (2, 2, 2), (5, 6, 8)), "S2_BACKWARD", 2, "Vy", 0.7),
                            (("sphere", 3, (3, 5, 7)), "P_FORWARD", 1, "PRESSURE", -1.0)],
                     quantities=[(("infinite",), "Syz", 0.3)]),
    "two_bodies_2d": spec(2, 2, [1, 0.25], {0: ([21, 41], [0, 0]), 1: ([21, 41], [0, 41])}, 0.9,
                          (4, 2, 0.5), snaps=1,
                          waves=[(("box", (-1000, 2.5, -1000), (1000, 7.5, 1000)), "P_FORWARD", 1,
                                  "PRESSURE", 1.0),
                                 (("box", (3, 9, -1), (9, 12, 1)), "S1_BACKWARD", 0, "Sxy", 0.25)]),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_host_state_matches_oracle(H, name):
    s = CASES[name]
    oe = O.Engine(oracle_task(s))
    ht = host_task(s)
    for b in oe.bodies:
        st = H.host_state(ht, b.id)
        pde = st["pde"]
        assert pde.shape == b.shape_all + (b.M,)
        want = b.pde.reshape(pde.shape)
        assert np.array_equal(pde, want), f"{int((pde != want).sum())} values differ"
        # +0.0 vs -0.0 as well (initial conditions are sums of signed terms)
        assert np.array_equal(np.signbit(pde), np.signbit(want))
        assert np.array_equal(st["mat_ids"], b.mat_id.reshape(b.shape_all))
        assert st["maximal_eigenvalue"] == b.maximal_eigenvalue
        assert st["n_conditions"] == len(b.tables)


def test_host_state_errors(H):
    s = spec(3, 2, [1, 1, 1], {0: ([6, 6, 6], [0, 0, 0])}, 0.9, (4, 2, 1), snaps=1,
             vectors=[(("infinite",), [1.0, 2.0])])
    with pytest.raises(H.GcmException):
        H.host_state(host_task(s), 0)
    s = spec(2, 2, [1, 1], {0: ([6, 6], [0, 0])}, 0.9, (4, 2, 1), snaps=1,
             waves=[(("infinite",), "P_FORWARD", 2, "Vx", 1.0)])
    with pytest.raises(H.GcmException):
        H.host_state(host_task(s), 0)
    s = spec(2, 2, [1, 1], {0: ([6, 6], [0, 0])}, 0.9, (4, 2, 1), snaps=1)
    with pytest.raises(Exception):
        H.host_state(host_task(s), 7)  # no such body
