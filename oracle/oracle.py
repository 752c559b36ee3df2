"""ctypes bindings of the CPU oracle (oracle/rt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


class _Scene(ctypes.Structure):
    _fields_ = [
        ("vp", ctypes.c_void_p), ("vn", ctypes.c_void_p), ("vuv", ctypes.c_void_p),
        ("face", ctypes.c_void_p), ("triCount", ctypes.c_int32),
        ("mat", ctypes.c_void_p), ("nmat", ctypes.c_int32),
        ("bvh", ctypes.c_void_p), ("nbvh_nodes", ctypes.c_int64),
        ("ibl", ctypes.c_void_p), ("ibl_w", ctypes.c_int32), ("ibl_h", ctypes.c_int32),
    ]


class _Counts(ctypes.Structure):
    _fields_ = [("nodes", ctypes.c_uint64), ("tris", ctypes.c_uint64), ("rays", ctypes.c_uint64),
                ("env", ctypes.c_uint64), ("dropped", ctypes.c_uint64)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        path = os.environ.get("ENSEM3A_ORACLE_LIB")   # the sanitizer build (tools/sanitize.sh)
        if not path:
            path = _LIB_PATH
            if not os.path.exists(path):
                build()
        _lib = ctypes.CDLL(path)
        _lib.oracle_render.restype = ctypes.c_int
        _lib.oracle_render.argtypes = [ctypes.POINTER(_Scene), ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                       ctypes.POINTER(_Counts)]
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


class OracleScene:
    """Keeps the numpy arrays alive for the C struct that points into them."""

    def __init__(self, V_p, V_n, V_uv, faceData, materialData, bvh, ibl_rgba):
        self.V_p = np.ascontiguousarray(V_p, dtype=np.float32)
        self.V_n = np.ascontiguousarray(V_n, dtype=np.float32)
        self.V_uv = np.ascontiguousarray(V_uv, dtype=np.float32) if V_uv is not None and len(V_uv) else None
        self.face = np.ascontiguousarray(faceData, dtype=np.int32)
        self.mat = np.ascontiguousarray(materialData, dtype=np.float32)
        self.bvh = np.ascontiguousarray(bvh, dtype=np.float32)
        ibl = np.ascontiguousarray(ibl_rgba, dtype=np.uint8)
        assert ibl.ndim == 3 and ibl.shape[2] == 4, "IBL must be HxWx4 RGBA8"
        self.ibl = ibl
        self.c = _Scene(_ptr(self.V_p), _ptr(self.V_n), _ptr(self.V_uv), _ptr(self.face),
                        self.face.size // 10, _ptr(self.mat), self.mat.size // 6,
                        _ptr(self.bvh), self.bvh.size // 9, _ptr(self.ibl), ibl.shape[1], ibl.shape[0])

    @classmethod
    def from_scene(cls, scene, ibl_rgba):
        return cls(scene.V_p, scene.V_n, scene.V_uv, scene.faceData, scene.materialData,
                   scene.BVH.exportArray, ibl_rgba)


def render(osc: OracleScene, cam, env, npix: int, spp: int, max_bounce: int, row0: int = 0,
           row_step: int = 1, nthreads: int = 0, counts: bool = False):
    """Render rows ``row0, row0+row_step, ...``; returns float32 [nrows*W*3] (and counters)."""
    cam = np.ascontiguousarray(cam, dtype=np.float32)
    env = np.ascontiguousarray(env, dtype=np.float32)
    W = int(cam[6])
    H = (npix + W - 1) // W
    nrows = max(0, (H - row0 + row_step - 1) // row_step)
    out = np.zeros(nrows * W * 3, dtype=np.float32)
    if nthreads <= 0:
        nthreads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cnt = _Counts()
    n = lib().oracle_render(ctypes.byref(osc.c), cam.ctypes.data, env.ctypes.data, npix, spp, max_bounce,
                            row0, row_step, nthreads, out.ctypes.data, ctypes.byref(cnt) if counts else None)
    if n < 0:
        raise ValueError("oracle_render: bad arguments")
    if counts:
        return out, dict(nodes=cnt.nodes, tris=cnt.tris, rays=cnt.rays, env=cnt.env, dropped=cnt.dropped)
    return out


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def rand_stream(seed0: int, seed1: int, n: int):
    out = np.zeros(n, np.float32)
    st = np.zeros(2, np.uint32)
    lib().oracle_rand_stream(ctypes.c_uint32(seed0), ctypes.c_uint32(seed1), ctypes.c_int(n),
                             ctypes.c_void_p(out.ctypes.data), ctypes.c_void_p(st.ctypes.data))
    return out, (int(st[0]), int(st[1]))


def camera_ray(cam, i: int):
    cam = _f32(cam)
    out = np.zeros(6, np.float32)
    lib().oracle_camera_ray(ctypes.c_void_p(cam.ctypes.data), ctypes.c_int(i), ctypes.c_void_p(out.ctypes.data))
    return out


def rotate(angle: float, axis, v):
    axis, v = _f32(axis), _f32(v)
    out = np.zeros(3, np.float32)
    lib().oracle_rotate(ctypes.c_float(angle), ctypes.c_void_p(axis.ctypes.data), ctypes.c_void_p(v.ctypes.data),
                        ctypes.c_void_p(out.ctypes.data))
    return out


def intersect(tri9, ray6):
    tri9, ray6 = _f32(tri9), _f32(ray6)
    out = np.zeros(2, np.float32)
    lib().oracle_intersect(ctypes.c_void_p(tri9.ctypes.data), ctypes.c_void_p(ray6.ctypes.data),
                           ctypes.c_void_p(out.ctypes.data))
    return out


def box(ray6, box6) -> bool:
    ray6, box6 = _f32(ray6), _f32(box6)
    return bool(lib().oracle_box(ctypes.c_void_p(ray6.ctypes.data), ctypes.c_void_p(box6.ctypes.data)))


def trace(osc: OracleScene, ray6):
    ray6 = _f32(ray6)
    out = np.zeros(8, np.float32)
    lib().oracle_trace(ctypes.byref(osc.c), ctypes.c_void_p(ray6.ctypes.data), ctypes.c_void_p(out.ctypes.data))
    return out


def brdf_ggx(mat6, v, l, n):
    mat6, v, l, n = _f32(mat6), _f32(v), _f32(l), _f32(n)
    out = np.zeros(3, np.float32)
    lib().oracle_brdf_ggx(*[ctypes.c_void_p(a.ctypes.data) for a in (mat6, v, l, n, out)])
    return out


def sample_ibl(osc: OracleScene, d):
    d = _f32(d)
    out = np.zeros(3, np.float32)
    lib().oracle_sample_ibl(ctypes.byref(osc.c), ctypes.c_void_p(d.ctypes.data), ctypes.c_void_p(out.ctypes.data))
    return out


def spherical_map(d):
    d = _f32(d)
    out = np.zeros(2, np.float32)
    lib().oracle_spherical_map(ctypes.c_void_p(d.ctypes.data), ctypes.c_void_p(out.ctypes.data))
    return out


def hemi(kind: int, n, seeds):
    n = _f32(n)
    io = np.array(seeds, dtype=np.uint32)
    out = np.zeros(4, np.float32)
    lib().oracle_hemi(ctypes.c_int(kind), ctypes.c_void_p(n.ctypes.data), ctypes.c_void_p(io.ctypes.data),
                      ctypes.c_void_p(out.ctypes.data))
    return out, (int(io[0]), int(io[1]))


MATH_FN = {"sin": 0, "cos": 1, "tan": 2, "asin": 3, "acos": 4, "atan2": 5, "sqrt": 6, "div": 7}


def math(fn: str, x, y=None):
    x = _f32(x)
    y = _f32(np.zeros_like(x) if y is None else y)
    out = np.zeros_like(x)
    lib().oracle_math(ctypes.c_int(MATH_FN[fn]), ctypes.c_void_p(x.ctypes.data), ctypes.c_void_p(y.ctypes.data),
                      ctypes.c_void_p(out.ctypes.data), ctypes.c_int64(x.size))
    return out


def gamma(x):
    """ImgProcessing.cl:1-10 (powr(min(x,1), 2.2)), evaluated in float64 and rounded to float32;
    powr is implementation-defined, so comparisons against it carry a tolerance."""
    x = np.asarray(x, dtype=np.float32)
    return np.power(np.minimum(x, np.float32(1)).astype(np.float64), 2.2).astype(np.float32)


def rgb8(data, gamma_first: bool = False):
    """Output stage of FileManager.saveImg (FileManager.py:334-336): ``(data*255).astype('uint8')``
    on a float32 frame (the product is float32: numpy's weak Python-int promotion); optionally
    after the gamma kernel (main.py:96-97 pairs them, commented out in the reference)."""
    d = np.asarray(data, dtype=np.float32)
    if gamma_first:
        d = gamma(d)
    return (d * 255).astype("uint8")


def pixel_log(osc: OracleScene, cam, env, npix: int, spp: int, max_bounce: int, pixel: int, cap: int = 4096):
    cam, env = _f32(cam), _f32(env)
    log = np.zeros((cap, 16), np.float32)
    out3 = np.zeros(3, np.float32)
    n = lib().oracle_pixel_log(ctypes.byref(osc.c), ctypes.c_void_p(cam.ctypes.data), ctypes.c_void_p(env.ctypes.data),
                               ctypes.c_int32(npix), ctypes.c_int32(spp), ctypes.c_int32(max_bounce),
                               ctypes.c_int32(pixel), ctypes.c_void_p(log.ctypes.data), ctypes.c_int32(cap),
                               ctypes.c_void_p(out3.ctypes.data))
    return log[:n].copy(), out3
