"""Measurement plumbing on the GPU: the STREAM-like copy that confirms the HBM
peak on the box, reported by bench.py next to the 8 TB/s spec."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu


def test_hbm_copy_bandwidth_is_plausible():
    from tt2 import _lib
    lib = _lib.load_library()
    g = ctypes.c_double(0.0)
    _lib.check(lib.tt2_hbm_copy_gbps(0, ctypes.c_longlong(1 << 28), 3, ctypes.byref(g)))
    # a float4 copy reaches ~6.3 TB/s on MI355X (MI355X_MICROARCH.md); never above the 8 TB/s spec
    assert 2000.0 < g.value < 8200.0, g.value


def test_hbm_copy_rejects_bad_arguments():
    from tt2 import _lib
    lib = _lib.load_library()
    g = ctypes.c_double(0.0)
    assert lib.tt2_hbm_copy_gbps(0, ctypes.c_longlong(1024), 3, ctypes.byref(g)) != 0
    assert lib.tt2_hbm_copy_gbps(0, ctypes.c_longlong(1 << 24), 0, ctypes.byref(g)) != 0
