"""Drive the reference's own OpenCL kernels on the ROCm OpenCL runtime.

TEST INFRASTRUCTURE ONLY (golden-fixture generation, tools/gen_golden.py).
Needs oracle/_ref/ built by ``make -C oracle ref`` in the container that has
the reference tree; the binaries travel to the GPU box, the sources do not.

:func:`render` mirrors ``KernelLauncher.launch_Raytracing``
(KernelLauncher.py:33-87): same buffers, same scalar arguments, same global
size, local size left to the runtime.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(_HERE, "_ref")
RT_CO = os.path.join(REF_DIR, "raytracing_gfx950.co")
KAT_CO = os.path.join(REF_DIR, "kat_gfx950.co")
_LIB = os.path.join(REF_DIR, "librefcl.so")
_lib = None
_open = None

_c = ctypes.c_void_p


def available() -> bool:
    return all(os.path.exists(p) for p in (RT_CO, KAT_CO, _LIB))


def _L():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(_LIB)
        _lib.refcl_error.restype = ctypes.c_char_p
        _lib.refcl_open.argtypes = [ctypes.c_char_p]
        _lib.refcl_kernel.argtypes = [ctypes.c_char_p]
        _lib.refcl_arg_buf.argtypes = [ctypes.c_int, ctypes.c_int, _c, ctypes.c_size_t, ctypes.c_int]
        _lib.refcl_arg_scalar.argtypes = [ctypes.c_int, ctypes.c_int, _c, ctypes.c_size_t]
        _lib.refcl_arg_image.argtypes = [ctypes.c_int, ctypes.c_int, _c, ctypes.c_int, ctypes.c_int]
        _lib.refcl_run.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_double)]
    return _lib


def _chk(st):
    if st < 0:
        raise RuntimeError("refcl: " + _L().refcl_error().decode(errors="replace"))
    return st


def open_program(path: str) -> None:
    global _open
    if _open == path:
        return
    if _open is not None:
        _L().refcl_close()
    _chk(_L().refcl_open(path.encode()))
    _open = path


def device_name() -> str:
    buf = ctypes.create_string_buffer(256)
    _L().refcl_device_name(buf, 256)
    return buf.value.decode(errors="replace")


class _Launch:
    def __init__(self, name: str):
        self.k = _chk(_L().refcl_kernel(name.encode()))
        self._keep = []

    def buf(self, idx: int, arr: np.ndarray, readback: bool = False):
        arr = np.array(arr, order="C", copy=True) if readback else np.ascontiguousarray(arr)
        self._keep.append(arr)
        _chk(_L().refcl_arg_buf(self.k, idx, arr.ctypes.data if arr.size else None, arr.nbytes, int(readback)))
        return arr

    def scalar(self, idx: int, value, ctype=ctypes.c_int):
        v = ctype(value)
        self._keep.append(v)
        _chk(_L().refcl_arg_scalar(self.k, idx, ctypes.byref(v), ctypes.sizeof(v)))

    def image(self, idx: int, rgba: np.ndarray):
        img = np.ascontiguousarray(rgba, dtype=np.uint8)
        self._keep.append(img)
        _chk(_L().refcl_arg_image(self.k, idx, img.ctypes.data, img.shape[1], img.shape[0]))

    def run(self, global_size: int) -> float:
        ms = ctypes.c_double(0.0)
        _chk(_L().refcl_run(self.k, global_size, ctypes.byref(ms)))
        return ms.value


def render(vp, vn, vuv, face, light, mat, bvh, cam, env, imgDim: int, spp: int, max_bounce: int, ibl_rgba):
    """Reference render; returns (float32 [3*imgDim], kernel milliseconds)."""
    open_program(RT_CO)
    out = np.zeros(3 * imgDim, dtype=np.float32)
    light = np.asarray(light, dtype=np.int32)
    if light.size == 0:
        light = np.array([0], dtype=np.int32)  # KernelLauncher.py:64-66
    L = _Launch("Raytracing")
    out = L.buf(0, out, readback=True)
    L.buf(1, np.asarray(vp, np.float32))
    L.buf(2, np.asarray(vn, np.float32))
    L.buf(3, np.asarray(vuv, np.float32))
    face = np.asarray(face, np.int32)
    L.buf(4, face)
    L.buf(5, light)
    L.buf(6, np.asarray(mat, np.float32))
    L.buf(7, np.asarray(bvh, np.float32))
    L.buf(8, np.asarray(cam, np.float32))
    L.buf(9, np.asarray(env, np.float32))
    L.scalar(10, face.size // 10, ctypes.c_uint32)
    L.scalar(11, int(np.asarray(light).size), ctypes.c_uint32)
    L.scalar(12, imgDim, ctypes.c_uint32)
    L.scalar(13, spp, ctypes.c_uint32)
    L.scalar(14, max_bounce, ctypes.c_uint32)
    L.image(15, ibl_rgba)
    ms = L.run(imgDim)
    return out, ms


# ---------------- known-answer tests of single reference functions ----------------

def _kat():
    open_program(KAT_CO)


def kat_rand(seeds: np.ndarray, nd: int):
    _kat()
    seeds = np.ascontiguousarray(seeds, np.uint32).reshape(-1, 2)
    n = seeds.shape[0]
    L = _Launch("kat_rand")
    L.buf(0, seeds.reshape(-1))
    L.scalar(1, nd)
    out = L.buf(2, np.zeros(n * nd, np.float32), True)
    st = L.buf(3, np.zeros(2 * n, np.uint32), True)
    L.run(n)
    return out.reshape(n, nd), st.reshape(n, 2)


def kat_camera(cam, idx):
    _kat()
    idx = np.ascontiguousarray(idx, np.int32)
    L = _Launch("kat_camera")
    L.buf(0, np.asarray(cam, np.float32))
    L.buf(1, idx)
    out = L.buf(2, np.zeros(6 * idx.size, np.float32), True)
    L.run(idx.size)
    return out.reshape(-1, 6)


def _simple(name, inp, width_in, width_out, out_dtype=np.float32):
    _kat()
    inp = np.ascontiguousarray(inp, np.float32).reshape(-1, width_in)
    n = inp.shape[0]
    L = _Launch(name)
    L.buf(0, inp.reshape(-1))
    out = L.buf(1, np.zeros(n * width_out, out_dtype), True)
    L.run(n)
    return out.reshape(n, width_out)


def kat_rotate(inp7):
    return _simple("kat_rotate", inp7, 7, 3)


def kat_intersect(inp15):
    return _simple("kat_intersect", inp15, 15, 2)


def kat_box(inp12):
    return _simple("kat_box", inp12, 12, 1, np.int32)[:, 0]


def kat_ggx(inp15):
    return _simple("kat_ggx", inp15, 15, 3)


def kat_trace(vp, vn, vuv, face, bvh, rays):
    _kat()
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    n = rays.shape[0]
    face = np.asarray(face, np.int32)
    L = _Launch("kat_trace")
    L.buf(0, np.asarray(vp, np.float32))
    L.buf(1, np.asarray(vn, np.float32))
    L.buf(2, np.asarray(vuv, np.float32))
    L.buf(3, face)
    L.buf(4, np.asarray(bvh, np.float32))
    L.scalar(5, face.size // 10)
    L.buf(6, rays.reshape(-1))
    out = L.buf(7, np.zeros(8 * n, np.float32), True)
    L.run(n)
    return out.reshape(n, 8)


def kat_ibl(ibl_rgba, dirs):
    _kat()
    dirs = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
    n = dirs.shape[0]
    L = _Launch("kat_ibl")
    L.image(0, ibl_rgba)
    L.buf(1, dirs.reshape(-1))
    out = L.buf(2, np.zeros(5 * n, np.float32), True)
    L.run(n)
    return out.reshape(n, 5)


def kat_sphmap(dirs):
    return _simple("kat_sphmap", dirs, 3, 2)


def image_support() -> bool:
    """False on gfx950: the ROCm OpenCL runtime exposes no images there (clCreateImage -> -59)."""
    open_program(RT_CO)
    try:
        L = _Launch("Raytracing")
        L.image(15, np.zeros((1, 1, 4), np.uint8))
        return True
    except RuntimeError:
        return False


def kat_texel(ibl_rgba, xy):
    _kat()
    xy = np.ascontiguousarray(xy, np.int32).reshape(-1, 2)
    n = xy.shape[0]
    L = _Launch("kat_texel")
    L.image(0, ibl_rgba)
    L.buf(1, xy.reshape(-1))
    out = L.buf(2, np.zeros(4 * n, np.float32), True)
    L.run(n)
    return out.reshape(n, 4)


def kat_hemi(kind: int, normals, seeds):
    _kat()
    normals = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
    n = normals.shape[0]
    L = _Launch("kat_hemi")
    L.scalar(0, kind)
    L.buf(1, normals.reshape(-1))
    sd = L.buf(2, np.ascontiguousarray(seeds, np.uint32).reshape(-1), True)
    out = L.buf(3, np.zeros(4 * n, np.float32), True)
    L.run(n)
    return out.reshape(n, 4), sd.reshape(n, 2)


def kat_math(fn: int, x, y=None):
    _kat()
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, np.float32)
    L = _Launch("kat_math")
    L.scalar(0, fn)
    L.buf(1, x)
    L.buf(2, y)
    out = L.buf(3, np.zeros_like(x), True)
    L.run(x.size)
    return out
