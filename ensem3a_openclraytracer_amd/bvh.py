"""BVH export identical to the reference's ``BVH(faceData, V_p).exportArray``.

The reference builds it in pure Python (``BVH.py:120-191``, 336 s for 1M
triangles); here the same algorithm runs natively (``csrc/bvh_build.cpp``)
and reproduces the export bit for bit (pinned by the hashes in
``tests/golden/bvh_hashes.json``).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native


class DegenerateBVHError(ValueError):
    """The reference builder would not terminate on this input (duplicate centroids)."""


def build_export_array(faceData, V_p) -> np.ndarray:
    """float32 ``[9 * (2T-1)]``: per node ``[left, right, min.xyz, max.xyz, tri | -1]``."""
    face = _native.i32(faceData).reshape(-1)
    vp = _native.f32(V_p).reshape(-1)
    if face.size % 10:
        raise ValueError("faceData length must be a multiple of 10")
    T = face.size // 10
    if T == 0:
        return np.zeros(0, dtype=np.float32)
    out = np.zeros(9 * (2 * T - 1), dtype=np.float32)
    nodes = ctypes.c_int64(0)
    st = _native.host_lib().rt_bvh_build(face.ctypes.data, face.size, vp.ctypes.data, vp.size, out.ctypes.data,
                                    ctypes.byref(nodes))
    if st == 3:
        raise DegenerateBVHError("a split left one side empty: the reference BVH.py would recurse forever "
                                 "(triangles with identical centroids)")
    if st == 2:
        raise ValueError("faceData position index out of range")
    if st == 4:
        raise MemoryError("rt_bvh_build: out of host memory")
    if st != 0:
        raise ValueError(f"rt_bvh_build failed with status {st}")
    return out[: 9 * nodes.value]


class BVH:
    """Drop-in for the reference ``BVH`` class: ``BVH(faceData, V_p).exportArray``."""

    def __init__(self, faceData, V_p):
        self.exportArray = build_export_array(faceData, V_p)
        self.NodeCounter = self.exportArray.size // 9
