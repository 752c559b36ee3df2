"""The C-ABI library: loads without a GPU, exports every declared symbol, and the
product path fails loudly (no CPU fallback) when no device is present."""
import ctypes
import os
import re

import numpy as np
import pytest

from ensem3a_openclraytracer_amd import _native
from ensem3a_openclraytracer_amd._build import LIB

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in ("rt_api.h", "rt_debug.h", "rt_scene.h"):
        with open(os.path.join(ROOT, "include", h)) as f:
            txt = f.read()
        names |= set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", txt))
    return names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    declared = _declared()
    assert declared == set(_native.EXPORTED), declared ^ set(_native.EXPORTED)
    for name in declared:
        assert hasattr(lib, name), name


def test_host_entry_points_without_gpu():
    assert _native.tile_rows(1024 * 1024, 1024, 0, 1) == 1024
    assert _native.tile_rows(10, 4, 1, 2) == 1          # rows 0..2, tile 1::2 -> row 1
    assert _native.tile_rows(10, 4, 5, 2) == 0
    assert _native.tile_rows(0, 4, 0, 1) == 0


@pytest.mark.skipif(_native.device_count() > 0, reason="a GPU is present")
def test_no_gpu_raises_loudly():
    with pytest.raises(_native.NativeError, match="no HIP device"):
        _native.Context()
    from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher
    with pytest.raises(RuntimeError):
        KernelLauncher(None, None, None, None)


def test_missing_library_is_an_error(monkeypatch):
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB", "/nonexistent/libensem3a_rt.so")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _native.lib()


def test_bvh_through_abi_validates():
    from ensem3a_openclraytracer_amd.bvh import build_export_array
    with pytest.raises(ValueError):
        build_export_array(np.array([0] * 7 + [5, 6, 7], np.int32), np.zeros(9, np.float32))
