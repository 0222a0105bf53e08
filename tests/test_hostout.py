"""HostOut: the host array a solve's iterate is downloaded into, its pages
faulted in by a helper thread while the device iterates (krylov_amd/device.py).
Host logic only: no device call."""
import numpy as np


def test_hostout_large_is_prefaulted_and_usable():
    from krylov_amd.device import HostOut

    h = HostOut((3_000_000, 1), np.float64)  # 24 MB: above MIN_BYTES (8 MiB), so a helper thread runs
    assert h._t is not None
    a = h.take()
    assert h._t is None and a.shape == (3_000_000, 1) and a.dtype == np.float64 and a.flags.c_contiguous
    assert not a.any()  # the helper wrote zeros over every page
    assert h.take() is a  # joining twice is harmless


def test_hostout_small_has_no_thread():
    from krylov_amd.device import HostOut

    h = HostOut((1000, 4), np.float32)
    assert h._t is None
    a = h.take()
    assert a.shape == (1000, 4) and a.dtype == np.float32
