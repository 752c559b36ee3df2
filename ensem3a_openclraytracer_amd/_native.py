"""ctypes binding of the native library ``lib/libensem3a_rt.so`` (include/rt_api.h).

There is no fallback: if the library is missing or fails to load, every entry
point raises.  The library is built in-tree by ``_build.build()``.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

from ._build import LIB

_lock = threading.Lock()
_lib = None
_host = None

RT_TRAVERSAL_FAST = 0
RT_TRAVERSAL_REF = 1
RT_BVH_REFERENCE = 0
RT_BVH_SAH = 1

# Every symbol of include/rt_api.h and include/rt_debug.h (checked by tests).
EXPORTED = (
    "rt_create", "rt_destroy", "rt_last_error", "rt_set_scene", "rt_set_env", "rt_set_option",
    "rt_render", "rt_render_device", "rt_tile_rows", "rt_count_work", "rt_count_work_detail", "rt_work_bytes", "rt_gamma",
    "rt_render_rgb8", "rt_rgb8_device", "rt_rgb8",
    "rt_bvh_build", "rt_device_count", "rt_debug_math", "rt_debug_trace", "rt_debug_scene_info", "rt_debug_pixel_log",
    "rt_debug_wave_counts", "rt_debug_quantise_axis", "rt_debug_timings",
    "rt_obj_parse", "rt_obj_size", "rt_obj_copy", "rt_obj_free", "rt_obj_last_error",
    "rt_scene_check", "rt_scene_last_error",
)
# The host-only entry points (no GPU, no HIP call): the sanitizer build (oracle/Makefile asan,
# tools/sanitize.sh) compiles exactly these into an ASan/UBSan library that ENSEM3A_HOST_LIB selects.
HOST_ONLY = ("rt_bvh_build", "rt_obj_parse", "rt_obj_size", "rt_obj_copy", "rt_obj_free", "rt_obj_last_error",
             "rt_scene_check", "rt_scene_last_error", "rt_debug_quantise_axis")

_c_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int


class NativeError(RuntimeError):
    """A non-zero status from the native library (mirrors pyopencl raising)."""

    def __init__(self, status: int, message: str):
        super().__init__(f"[rt status {status}] {message}")
        self.status = status


def _preload_hip_runtime() -> None:
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    for d in (spec.submodule_search_locations or []) if spec else []:
        p = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(p):
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
            return


def lib():
    """Load (once) and return the native library; raise loudly when absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        # torch ships its own HIP runtime (torch/lib/libamdhip64.so, SONAME libamdhip64.so.7, the
        # same SONAME as ROCm's): whichever is loaded first serves the whole process, and torch
        # cannot initialise its GPUs on ROCm's.  So when torch is installed its runtime is loaded
        # first -- as a plain shared library, without importing torch: the single-GPU drop-in path
        # (KernelLauncher) needs no torch, and a torch imported later finds its own runtime
        # already loaded (tests/test_gpu_boundary.py).
        _preload_hip_runtime()
        lib_path = os.environ.get("ENSEM3A_RT_LIB", LIB)  # experimental variants (tools/variants.py)
        if not os.path.exists(lib_path):
            raise RuntimeError(
                f"native library {lib_path} is missing: build it with "
                "`python -m ensem3a_openclraytracer_amd._build` (there is no CPU fallback)")
        L = ctypes.CDLL(lib_path)
        sig = {
            "rt_create": (_i32, [_i32, _c_p, ctypes.POINTER(_c_p)]),
            "rt_destroy": (None, [_c_p]),
            "rt_last_error": (ctypes.c_char_p, [_c_p]),
            "rt_set_scene": (_i32, [_c_p, _c_p, _i64, _c_p, _i64, _c_p, _i64, _c_p, _i64, _c_p, _i64, _c_p, _i64]),
            "rt_set_env": (_i32, [_c_p, _c_p, _i32, _i32]),
            "rt_set_option": (_i32, [_c_p, ctypes.c_char_p, _i64]),
            "rt_render": (_i32, [_c_p, _c_p, _c_p, _i64, _i32, _i32, _c_p]),
            "rt_render_device": (_i32, [_c_p, _i32, _c_p, _c_p, _i64, _i32, _i32, _i32, _i32, _c_p, _c_p]),
            "rt_tile_rows": (_i64, [_i64, _i32, _i32, _i32]),
            "rt_count_work": (_i32, [_c_p, _c_p, _c_p, _i64, _i32, _i32, _i32, _i32, _c_p]),
            "rt_count_work_detail": (_i32, [_c_p, _c_p, _c_p, _i64, _i32, _i32, _i32, _i32, _c_p]),
            "rt_work_bytes": (_i32, [_c_p, _c_p]),
            "rt_gamma": (_i32, [_c_p, _c_p, _c_p, _i64]),
            "rt_render_rgb8": (_i32, [_c_p, _c_p, _c_p, _i64, _i32, _i32, _i32, _c_p]),
            "rt_rgb8_device": (_i32, [_c_p, _i32, _c_p, _c_p, _i64, _i32, _c_p]),
            "rt_rgb8": (_i32, [_c_p, _c_p, _c_p, _i64, _i32]),
            "rt_bvh_build": (_i32, [_c_p, _i64, _c_p, _i64, _c_p, ctypes.POINTER(_i64)]),
            "rt_device_count": (_i32, []),
            "rt_obj_parse": (_i32, [_c_p, _i64, ctypes.POINTER(_c_p)]),
            "rt_obj_size": (_i64, [_c_p, _i32]),
            "rt_obj_copy": (_i32, [_c_p, _c_p, _c_p, _c_p, _c_p]),
            "rt_obj_free": (None, [_c_p]),
            "rt_obj_last_error": (ctypes.c_char_p, []),
            "rt_scene_check": (_i32, [_c_p, _i64, _c_p, _i64, _c_p, _i64, _c_p, _i64, _c_p, _i64, _i32, _c_p]),
            "rt_scene_last_error": (ctypes.c_char_p, []),
            "rt_debug_math": (_i32, [_c_p, _i32, _c_p, _c_p, _c_p, _i64]),
            "rt_debug_trace": (_i32, [_c_p, _i32, _c_p, _c_p, _i64]),
            "rt_debug_scene_info": (_i32, [_c_p, _c_p]),
            "rt_debug_timings": (_i32, [_c_p, _c_p]),
            "rt_debug_wave_counts": (_i32, [_c_p, _c_p, _c_p, _i64, _i32, _i32, _c_p]),
            "rt_debug_pixel_log": (_i32, [_c_p, _i32, _c_p, _c_p, _i64, _i32, _i32, _i64, _c_p, _i32, _c_p, _c_p]),
        }
        _bind(L, sig)
        _lib = L
    return _lib


_HOST_SIG = {}


def _bind(L, sig, names=None):
    for name, (res, args) in sig.items():
        if names is not None and name not in names:
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
        if name in HOST_ONLY:
            _HOST_SIG[name] = (res, args)


def host_lib():
    """The library serving the host-only entry points (HOST_ONLY): the product library, or the
    sanitizer build named by ENSEM3A_HOST_LIB (tools/sanitize.sh)."""
    global _host
    if _host is not None:
        return _host
    L = lib()
    path = os.environ.get("ENSEM3A_HOST_LIB")
    if path:
        with _lock:
            if _host is None:
                H = ctypes.CDLL(path)
                _bind(H, _HOST_SIG)
                _host = H
        return _host
    _host = L
    return _host


def check(status: int, ctx=None) -> None:
    if status != 0:
        msg = lib().rt_last_error(ctx)
        raise NativeError(status, msg.decode(errors="replace") if msg else "unknown error")


def f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


def ptr(a: np.ndarray):
    return a.ctypes.data if a is not None and a.size else None


def device_count() -> int:
    return int(lib().rt_device_count())


class Context:
    """Owner of one ``rt_ctx`` (one per host thread)."""

    def __init__(self, n_devices: int = 1, device_ids=None):
        ids = None
        if device_ids is not None:
            ids = (ctypes.c_int * len(device_ids))(*device_ids)
            n_devices = len(device_ids)
        out = _c_p()
        check(lib().rt_create(int(n_devices), ids, ctypes.byref(out)))
        self._ctx = out
        self.n_devices = int(n_devices)

    @property
    def handle(self):
        if self._ctx is None:
            raise RuntimeError("context destroyed")
        return self._ctx

    def close(self) -> None:
        if getattr(self, "_ctx", None) is not None:
            lib().rt_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int) -> None:
        check(st, self.handle)

    def set_option(self, key: str, value: int) -> None:
        self._check(lib().rt_set_option(self.handle, key.encode(), int(value)))

    def set_scene(self, V_p, V_n, V_uv, faceData, materialData, bvh) -> None:
        vp, vn, vuv = f32(V_p), f32(V_n), f32(V_uv if V_uv is not None else np.zeros(0, np.float32))
        face, mat, bv = i32(faceData), f32(materialData), f32(bvh)
        self._check(lib().rt_set_scene(self.handle, ptr(vp), vp.size, ptr(vn), vn.size, ptr(vuv), vuv.size,
                                       ptr(face), face.size, ptr(mat), mat.size, ptr(bv), bv.size))

    def set_env(self, rgba: np.ndarray) -> None:
        img = np.ascontiguousarray(rgba, dtype=np.uint8)
        if img.ndim != 3 or img.shape[2] != 4:
            raise ValueError(f"IBL must be an HxWx4 RGBA8 array, got shape {img.shape}")
        self._check(lib().rt_set_env(self.handle, ptr(img), img.shape[1], img.shape[0]))

    def render(self, cam, env, npix: int, spp: int, max_bounce: int, out: np.ndarray = None) -> np.ndarray:
        c, e = f32(cam), f32(env)
        if c.size != 10 or e.size != 5:
            raise ValueError("cam must have 10 floats and envData 5")
        if out is None:
            out = np.zeros(3 * int(npix), dtype=np.float32)
        if out.dtype != np.float32 or not out.flags.c_contiguous or out.size < 3 * int(npix):
            raise ValueError("output must be a contiguous float32 array of 3*imgDim elements")
        self._check(lib().rt_render(self.handle, ptr(c), ptr(e), int(npix), int(spp), int(max_bounce),
                                    out.ctypes.data))
        return out

    def render_device(self, cam, env, npix, spp, max_bounce, row0, row_step, d_out_ptr: int, stream_ptr: int = 0,
                      device_index: int = 0) -> None:
        c, e = f32(cam), f32(env)
        self._check(lib().rt_render_device(self.handle, int(device_index), ptr(c), ptr(e), int(npix), int(spp),
                                           int(max_bounce), int(row0), int(row_step), _c_p(int(d_out_ptr)),
                                           _c_p(int(stream_ptr)) if stream_ptr else None))  # 0 = default stream

    def count_work(self, cam, env, npix, spp, max_bounce, row0=0, row_step=1):
        c, e = f32(cam), f32(env)
        out = np.zeros(5, dtype=np.uint64)
        self._check(lib().rt_count_work(self.handle, ptr(c), ptr(e), int(npix), int(spp), int(max_bounce),
                                        int(row0), int(row_step), out.ctypes.data))
        return dict(zip(("node_fetches", "tri_tests", "rays", "env_lookups", "stack_drops"), map(int, out)))

    COUNT_KEYS = ("node_fetches", "tri_tests", "rays", "env_lookups", "stack_drops", "wave_trav_iters",
                  "wave_render_iters", "cycles_shade", "cycles_trav", "box_tests", "ev_diffuse", "ev_glossy",
                  "ev_glass", "sun_terms", "samples")

    def count_work_detail(self, cam, env, npix, spp, max_bounce, row0=0, row_step=1):
        """rt_count_work_detail: every work counter of the instrumented render of the tile."""
        c, e = f32(cam), f32(env)
        out = np.zeros(16, dtype=np.uint64)
        self._check(lib().rt_count_work_detail(self.handle, ptr(c), ptr(e), int(npix), int(spp), int(max_bounce),
                                               int(row0), int(row_step), out.ctypes.data))
        return {k: int(v) for k, v in zip(self.COUNT_KEYS, out)}

    def work_bytes(self):
        out = np.zeros(4, dtype=np.float64)
        self._check(lib().rt_work_bytes(self.handle, out.ctypes.data))
        return dict(zip(("box_test", "tri_test", "ray", "env_lookup"), map(float, out)))

    def gamma(self, src, out=None):
        s = f32(src)
        if out is None:
            out = np.zeros_like(s)
        self._check(lib().rt_gamma(self.handle, ptr(s), out.ctypes.data, s.size))
        return out

    def render_rgb8(self, cam, env, npix: int, spp: int, max_bounce: int, gamma: bool = False,
                    out: np.ndarray = None) -> np.ndarray:
        """Render and quantize on the device: uint8[3*npix] = (frame*255).astype(uint8) (gamma first if asked)."""
        c, e = f32(cam), f32(env)
        if c.size != 10 or e.size != 5:
            raise ValueError("cam must have 10 floats and envData 5")
        if out is None:
            out = np.zeros(3 * int(npix), dtype=np.uint8)
        if out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < 3 * int(npix):
            raise ValueError("output must be a contiguous uint8 array of 3*imgDim elements")
        self._check(lib().rt_render_rgb8(self.handle, ptr(c), ptr(e), int(npix), int(spp), int(max_bounce),
                                         int(bool(gamma)), out.ctypes.data))
        return out

    def rgb8(self, src, gamma: bool = False, out=None) -> np.ndarray:
        """Host float32 -> uint8 through the device output stage."""
        s = f32(src).reshape(-1)
        if out is None:
            out = np.zeros(s.size, dtype=np.uint8)
        self._check(lib().rt_rgb8(self.handle, ptr(s), out.ctypes.data, s.size, int(bool(gamma))))
        return out

    def rgb8_device(self, d_in_ptr: int, d_out_ptr: int, n: int, gamma: bool = False, stream_ptr: int = 0,
                    device_index: int = 0) -> None:
        self._check(lib().rt_rgb8_device(self.handle, int(device_index), _c_p(int(d_in_ptr)), _c_p(int(d_out_ptr)),
                                         int(n), int(bool(gamma)), _c_p(int(stream_ptr)) if stream_ptr else None))

    def debug_math(self, fn: int, x, y=None):
        x = f32(x)
        yy = f32(y) if y is not None else None
        out = np.zeros_like(x)
        self._check(lib().rt_debug_math(self.handle, int(fn), ptr(x), ptr(yy), out.ctypes.data, x.size))
        return out

    def debug_trace(self, rays, traversal: int):
        r = f32(rays).reshape(-1)
        out = np.zeros(2 * (r.size // 6), dtype=np.float32)
        self._check(lib().rt_debug_trace(self.handle, int(traversal), ptr(r), out.ctypes.data, r.size // 6))
        return out.reshape(-1, 2)

    def debug_pixel_log(self, traversal, cam, env, npix, spp, max_bounce, pixel, cap=4096):
        c, e = f32(cam), f32(env)
        log = np.zeros((cap, 16), np.float32)
        n = ctypes.c_int(0)
        out3 = np.zeros(3, np.float32)
        self._check(lib().rt_debug_pixel_log(self.handle, int(traversal), ptr(c), ptr(e), int(npix), int(spp),
                                             int(max_bounce), int(pixel), log.ctypes.data, cap, ctypes.byref(n),
                                             out3.ctypes.data))
        return log[: n.value].copy(), out3

    def wave_counts(self, cam, env, npix, spp, max_bounce):
        """rt_debug_wave_counts: lane counters + wave-level loop iterations of one frame."""
        c, e = f32(cam), f32(env)
        out = np.zeros(9, dtype=np.uint64)
        self._check(lib().rt_debug_wave_counts(self.handle, ptr(c), ptr(e), int(npix), int(spp), int(max_bounce),
                                               out.ctypes.data))
        keys = ("node_fetches", "tri_tests", "rays", "env_lookups", "stack_drops", "wave_trav_iters",
                "wave_render_iters", "cycles_shade", "cycles_trav")
        return {k: int(v) for k, v in zip(keys, out)}

    def scene_info(self):
        out = np.zeros(8, dtype=np.int64)
        self._check(lib().rt_debug_scene_info(self.handle, out.ctypes.data))
        return dict(fast_ok=bool(out[0]), depth=int(out[1]), nodes=int(out[2]), tris=int(out[3]),
                    brute_records=int(out[4]), brute_boxes=int(out[5]), wdq_omax=int(out[6]) * 1e-6)

    def timings(self) -> dict:
        """Host wall times (ms) of the last set_scene (pack / upload), set_env and render (rt_debug_timings)."""
        out = np.zeros(4, dtype=np.float64)
        self._check(lib().rt_debug_timings(self.handle, out.ctypes.data))
        return dict(pack_ms=float(out[0]), upload_ms=float(out[1]), env_ms=float(out[2]), render_ms=float(out[3]))


def parse_obj(text):
    """Native OBJ import (include/rt_scene.h): ``(V_p, V_n, V_uv, faceData, matCounter)``
    with the reference importer's semantics (FileManager.py:253-304).  Host only."""
    data = text.encode() if isinstance(text, str) else bytes(text)
    h = _c_p()
    H = host_lib()
    if H.rt_obj_parse(data, len(data), ctypes.byref(h)) != 0:
        raise ValueError("OBJ parse failed: " + H.rt_obj_last_error().decode(errors="replace"))
    try:
        n = [int(H.rt_obj_size(h, k)) for k in range(5)]
        vp, vn, vuv = (np.zeros(n[k], np.float32) for k in range(3))
        face = np.zeros(n[3], np.int32)
        H.rt_obj_copy(h, vp.ctypes.data, vn.ctypes.data, vuv.ctypes.data, face.ctypes.data)
    finally:
        H.rt_obj_free(h)
    return vp, vn, vuv, face, n[4]


def scene_check(V_p, V_n, faceData, materialData, bvh, layout: int = RT_BVH_SAH) -> dict:
    """rt_scene_check (include/rt_scene.h): the validation and repacking rt_set_scene applies, on the
    host alone (no GPU).  Raises NativeError with rt_set_scene's status for arrays it would refuse;
    returns the packed layout's sizes and, when the FAST layouts are unavailable, why."""
    vp, vn, face, mat, b = f32(V_p), f32(V_n), i32(faceData), f32(materialData), f32(bvh)
    info = np.zeros(8, np.int64)
    H = host_lib()
    st = H.rt_scene_check(ptr(vp), vp.size, ptr(vn), vn.size, ptr(face), face.size, ptr(mat), mat.size,
                          ptr(b), b.size, int(layout), info.ctypes.data)
    msg = H.rt_scene_last_error().decode(errors="replace")
    if st != 0:
        raise NativeError(st, msg)
    return dict(tris=int(info[0]), nodes=int(info[1]), depth=int(info[2]), wnodes=int(info[3]),
                wdepth=int(info[4]), brute_records=int(info[5]), brute_boxes=int(info[6]), fast_ok=bool(info[7]),
                note=msg)


def tile_rows(npix: int, width: int, row0: int, row_step: int) -> int:
    return int(lib().rt_tile_rows(int(npix), int(width), int(row0), int(row_step)))
