"""A layer larger than the 32-bit element space of one component plane.

520 x 1024 x 1024 nodes: 4.5 GB per component plane, 82 GB for the two
layers.  The one-pass step addresses each block's planes from bases at its own
plane (onepass_layout_ok), so such a grid runs the one-pass kernel
(k_fused_xyz, Z = 1024) rather than the generic stages.  Checked without
downloading the 82 GB: small probe contexts at corners, faces and the middle
of the grid hold the same parity-random field (fill_random is a function of
the GLOBAL node index), step on their own, and their nodes outside the
dependency radius of their own boundary (bs per stage and step) must equal the
big grid's, copied out with gcmx_copy_box, bitwise (exact floating-point mode:
both kernels keep the reference's operation order).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GX, GY, GZ = 520, 1024, 1024
NB = 16       # probe edge
STEPS = 2
BS = 2
MARGIN = BS * STEPS  # one step moves information bs nodes per axis


@pytest.mark.timeout(300)
def test_layer_over_4gb_per_plane_runs_one_pass_and_matches_probes():
    import gcm_amd
    from gcm_amd import gcmx
    from gcm_amd.host import isotropic_elastic_matrices
    U, U1, L = isotropic_elastic_matrices(3, 4.0, 2.0, 1.0)

    def ctx(sizes, start):
        c = gcm_amd.Context(3, BS, sizes, start=start)
        c.set_materials(U[None], U1[None], L[None])
        c.fp_mode = gcmx.FP_EXACT
        return c

    big = ctx([GX, GY, GZ], [0, 0, 0])
    try:
        assert big.effective_path == "fused"
        big.fill_random([GX, GY, GZ], 0xB16)
        for _ in range(STEPS):
            big.step(0.9)
        assert big.last_path == "fused"
        big.sync()
        probes = [(0, 0, 0), (GX - NB, GY - NB, GZ - NB), (GX // 2 - 5, GY // 2 + 3, GZ // 2 - 7),
                  (0, GY - NB, 500), (GX - NB, 0, GZ - NB), (250, 0, 0)]
        for p in probes:
            probe = ctx([NB] * 3, list(p))
            copy = ctx([NB] * 3, list(p))
            try:
                probe.fill_random([GX, GY, GZ], 0xB16)
                for _ in range(STEPS):
                    probe.step(0.9)
                copy.copy_box([0, 0, 0], [NB] * 3, big, list(p))
                a = probe.download().reshape(NB + 2 * BS, NB + 2 * BS, NB + 2 * BS, 9)
                b = copy.download().reshape(NB + 2 * BS, NB + 2 * BS, NB + 2 * BS, 9)
                sl = []
                for d, g in zip(p, (GX, GY, GZ)):
                    lo = 0 if d == 0 else MARGIN  # a probe face on the grid's face is exact
                    hi = NB if d + NB == g else NB - MARGIN
                    sl.append(slice(BS + lo, BS + hi))
                pa, pb = a[tuple(sl)], b[tuple(sl)]
                assert pa.size > 0 and np.abs(pa).sum() > 0
                assert np.array_equal(pa, pb), f"probe at {p}: {int((pa != pb).sum())} values differ"
            finally:
                probe.close()
                copy.close()
    finally:
        big.close()
