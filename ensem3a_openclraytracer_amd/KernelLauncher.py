"""Drop-in replacement of the reference's ``KernelLauncher`` (KernelLauncher.py:6-103).

Same constructor and method signatures, same argument meaning, same in-place
output contract; the pyopencl program build / buffer uploads / enqueue /
blocking read-back are replaced by ctypes calls into the HIP C-ABI
(include/rt_api.h).  Errors raise :class:`~._native.NativeError`
(a ``RuntimeError``), as pyopencl raises its own ``RuntimeError`` subclasses.
"""
from __future__ import annotations

from typing import Optional, Sequence, Union

import numpy as np

from . import _native

try:  # xxhash is in the image; hashlib is the portable fallback for the upload cache key
    import xxhash

    def _digest(a: np.ndarray) -> bytes:
        return xxhash.xxh3_128_digest(memoryview(np.ascontiguousarray(a)).cast("B"))
except ImportError:  # pragma: no cover
    import hashlib

    def _digest(a: np.ndarray) -> bytes:
        return hashlib.blake2b(memoryview(np.ascontiguousarray(a)).cast("B"), digest_size=16).digest()


def _ibl_rgba(h_IBL) -> np.ndarray:
    """RGBA8 texels of the IBL: a PIL image (as ``main.py:68`` passes) or an HxWx4 uint8 array."""
    if isinstance(h_IBL, np.ndarray):
        img = h_IBL
    elif hasattr(h_IBL, "tobytes") and hasattr(h_IBL, "size"):
        mode = getattr(h_IBL, "mode", "RGBA")
        if mode != "RGBA":
            h_IBL = h_IBL.convert("RGBA")
        w, h = h_IBL.size
        img = np.frombuffer(h_IBL.tobytes(), dtype=np.uint8).reshape(h, w, 4)
    else:
        raise TypeError("h_IBL must be a PIL.Image or an HxWx4 uint8 array")
    if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 4:
        raise ValueError(f"IBL must be RGBA8 (HxWx4 uint8), got {img.dtype} {img.shape}")
    return np.ascontiguousarray(img)


class KernelLauncher(object):
    """``KernelLauncher(context, platform, device, queue)``.

    ``context``, ``platform`` and ``queue`` exist for signature compatibility
    and are not used (there is no OpenCL context).  ``device`` selects the
    GPU(s): ``None`` = device 0, an ``int`` = that device, a sequence of ints =
    render on all of them (rows interleaved).  Keyword ``traversal`` picks the
    BVH traversal: ``"fast"`` (default) or ``"ref"`` (the reference's own DFS);
    ``bvh`` the tree the fast traversal walks: ``"sah"`` (default) or
    ``"reference"`` (the exported BVH.py tree) -- both give identical hits.
    """

    def __init__(self, context=None, platform=None, device: Union[None, int, Sequence[int]] = None, queue=None,
                 traversal: str = "fast", bvh: str = "sah"):
        self.platform = platform
        self.device = device
        self.context = context
        self.queue = queue
        if device is None or not isinstance(device, (int, list, tuple)):
            ids = [0]
        elif isinstance(device, int):
            ids = [device]
        else:
            ids = list(device)
        self._ctx = _native.Context(device_ids=ids)
        self.set_traversal(traversal)
        self.set_bvh(bvh)
        self._scene_key: Optional[tuple] = None
        self._env_key: Optional[tuple] = None

    def set_traversal(self, traversal: str) -> None:
        mode = {"fast": _native.RT_TRAVERSAL_FAST, "ref": _native.RT_TRAVERSAL_REF}.get(traversal)
        if mode is None:
            raise ValueError("traversal must be 'fast' or 'ref'")
        self._ctx.set_option("traversal", mode)
        self.traversal = traversal

    def set_bvh(self, bvh: str) -> None:
        mode = {"reference": _native.RT_BVH_REFERENCE, "sah": _native.RT_BVH_SAH}.get(bvh)
        if mode is None:
            raise ValueError("bvh must be 'sah' or 'reference'")
        self._ctx.set_option("bvh", mode)
        self.bvh = bvh

    @property
    def native(self) -> _native.Context:
        return self._ctx

    # ------------------------------------------------------------------
    def _upload_scene(self, vp, vn, vuv, face, mat, bvh) -> None:
        arrays = (_native.f32(vp), _native.f32(vn), _native.f32(vuv), _native.i32(face), _native.f32(mat),
                  _native.f32(bvh))
        key = tuple((a.size, _digest(a)) for a in arrays)
        if key != self._scene_key:
            self._ctx.set_scene(*arrays)
            self._scene_key = key

    def _upload_env(self, h_IBL) -> None:
        img = _ibl_rgba(h_IBL)
        key = (img.shape, _digest(img))
        if key != self._env_key:
            self._ctx.set_env(img)
            self._env_key = key

    def launch_Raytracing(self, h_img_out, h_vertex_p, h_vertex_n, h_vertex_uv, h_face_data, h_material_data,
                          h_light_data, h_BVH, h_cam, h_envData, imgDim, spp, maxBounce, h_IBL):
        """Render ``imgDim`` pixels into ``h_img_out`` (float32 ``[3*imgDim]``, written in place).

        Argument meaning as ``KernelLauncher.py:33-87``: the row width is
        ``int(h_cam[6])``; ``h_light_data`` is accepted and, as in the
        reference kernel, unused.  Blocking; returns ``None``.
        """
        if not isinstance(h_img_out, np.ndarray) or h_img_out.dtype != np.float32 or \
                not h_img_out.flags.c_contiguous:
            raise TypeError("h_img_out must be a C-contiguous float32 numpy array")
        imgDim = int(imgDim)
        if h_img_out.size < 3 * imgDim:
            raise ValueError(f"h_img_out has {h_img_out.size} floats, needs 3*imgDim = {3 * imgDim}")
        cam = _native.f32(h_cam).reshape(-1)
        env = _native.f32(h_envData).reshape(-1)
        if cam.size < 10 or env.size < 5:
            raise ValueError("h_cam needs 10 floats and h_envData 5")
        if h_light_data is not None:
            np.asarray(h_light_data)  # accepted for signature compatibility (unused by the kernel)
        self._upload_scene(h_vertex_p, h_vertex_n, h_vertex_uv, h_face_data, h_material_data, h_BVH)
        self._upload_env(h_IBL)
        out = h_img_out.reshape(-1)
        self._ctx.render(cam[:10], env[:5], imgDim, int(spp), int(maxBounce), out=out)

    def launch_Raytracing_rgb8(self, h_img_out, h_vertex_p, h_vertex_n, h_vertex_uv, h_face_data,
                               h_material_data, h_light_data, h_BVH, h_cam, h_envData, imgDim, spp, maxBounce,
                               h_IBL, gamma: bool = False):
        """``launch_Raytracing`` fused with the output stage: ``h_img_out`` is uint8 ``[3*imgDim]`` and
        receives ``(frame*255).astype('uint8')`` (FileManager.saveImg, FileManager.py:334-336),
        after the ImgProcessing gamma when ``gamma`` -- quantized on the device, so a quarter of
        the bytes cross PCIe."""
        if not isinstance(h_img_out, np.ndarray) or h_img_out.dtype != np.uint8 or \
                not h_img_out.flags.c_contiguous:
            raise TypeError("h_img_out must be a C-contiguous uint8 numpy array")
        imgDim = int(imgDim)
        if h_img_out.size < 3 * imgDim:
            raise ValueError(f"h_img_out has {h_img_out.size} bytes, needs 3*imgDim = {3 * imgDim}")
        cam = _native.f32(h_cam).reshape(-1)
        env = _native.f32(h_envData).reshape(-1)
        if cam.size < 10 or env.size < 5:
            raise ValueError("h_cam needs 10 floats and h_envData 5")
        self._upload_scene(h_vertex_p, h_vertex_n, h_vertex_uv, h_face_data, h_material_data, h_BVH)
        self._upload_env(h_IBL)
        self._ctx.render_rgb8(cam[:10], env[:5], imgDim, int(spp), int(maxBounce), gamma=gamma,
                              out=h_img_out.reshape(-1))

    def launch_ImgProcessing(self, h_src, h_out, SIZE):
        """Gamma 2.2 of ``ImgProcessing.cl``: ``h_out[k] = min(h_src[k], 1) ** 2.2`` for ``k < 3*SIZE*SIZE``."""
        src = _native.f32(h_src).reshape(-1)
        if not isinstance(h_out, np.ndarray) or h_out.dtype != np.float32 or not h_out.flags.c_contiguous:
            raise TypeError("h_out must be a C-contiguous float32 numpy array")
        n = min(int(SIZE) * int(SIZE) * 3, src.size, h_out.size)
        if n > 0:
            res = self._ctx.gamma(src[:n])
            h_out.reshape(-1)[:n] = res

    def close(self) -> None:
        self._ctx.close()
