"""Output stage and IBL input around the render.

* ``saveImg(data, sizeX, sizeY, name)`` -- FileManager.saveImg (FileManager.py:334-337):
  ``Image.fromarray((data*255).astype('uint8'), "RGB").save(name + ".png")``.  The
  quantization runs on the GPU (``rt_rgb8``, bit-identical to numpy's for rendered frames);
  PIL only encodes the PNG.
* ``to_rgb8(data, gamma)`` -- the quantization alone, optionally after the ImgProcessing.cl
  gamma (``launch_ImgProcessing``, KernelLauncher.py:90-103).
* ``load_ibl(path)`` -- ``Image.open(path).convert("RGBA")`` as main.py:68 does, returned as the
  RGBA8 texel array ``rt_set_env`` uploads (KernelLauncher.py:71-72 builds its cl.Image from
  the same bytes).
* ``scene_ibl(params, base_dir)`` -- the IBL a scene names in its ``IBLfile`` key (the
  reference's main.py ignores the key and always opens ``IBL/Arches_E_PineTree_8k.jpg``).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np

from . import _native

REFERENCE_IBL = "IBL/Arches_E_PineTree_8k.jpg"   # main.py:68


def _pil():
    try:
        from PIL import Image
    except ImportError as e:  # pragma: no cover - Pillow is part of the image
        raise RuntimeError("Pillow is required for PNG/JPEG I/O") from e
    return Image


def _context(launcher):
    if launcher is None:
        return _native.Context(device_ids=[0]), True
    return (launcher.native if hasattr(launcher, "native") else launcher), False


def to_rgb8(data, gamma: bool = False, launcher=None) -> np.ndarray:
    """uint8 array of ``data``'s shape: ``(data*255).astype('uint8')`` computed on the GPU."""
    arr = np.asarray(data, dtype=np.float32)
    ctx, own = _context(launcher)
    try:
        out = ctx.rgb8(arr.reshape(-1), gamma=gamma)
    finally:
        if own:
            ctx.close()
    return out.reshape(arr.shape)


def saveImg(data, sizeX: int, sizeY: int, name: str, launcher=None, gamma: bool = False) -> np.ndarray:
    """Write ``name + ".png"`` from a float frame (``[sizeX, sizeY, 3]`` or flat) or an already
    quantized uint8 frame; returns the uint8 ``[sizeX, sizeY, 3]`` image that was written."""
    arr = np.asarray(data)
    img = arr if arr.dtype == np.uint8 else to_rgb8(arr, gamma=gamma, launcher=launcher)
    img = np.ascontiguousarray(img).reshape(int(sizeX), int(sizeY), 3)
    _pil().fromarray(img, "RGB").save(name + ".png")
    return img


def load_ibl(path: str) -> np.ndarray:
    """RGBA8 texels ``[H, W, 4]`` of an image file (``Image.open(path).convert("RGBA")``)."""
    with _pil().open(path) as im:
        rgba = im.convert("RGBA")
        w, h = rgba.size
        return np.frombuffer(rgba.tobytes(), dtype=np.uint8).reshape(h, w, 4).copy()


def scene_ibl(params: Dict[str, str], base_dir: str, default: Optional[str] = REFERENCE_IBL) -> np.ndarray:
    """The IBL named by the scene's ``IBLfile`` key, relative to ``base_dir`` (the reference's
    working directory); ``default`` when the key is absent."""
    rel = params.get("IBLfile", default)
    if rel is None:
        raise KeyError("scene has no IBLfile key and no default was given")
    path = rel if os.path.isabs(rel) else os.path.join(base_dir, rel)
    if not os.path.exists(path):
        raise FileNotFoundError(f"IBL image {path} (IBLfile={rel!r}) does not exist")
    return load_ibl(path)
