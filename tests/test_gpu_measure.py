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
