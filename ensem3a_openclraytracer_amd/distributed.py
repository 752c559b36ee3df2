"""Multi-GPU rendering: one process per GPU, row-interleaved tiles, one gather.

Pixels are independent and the RNG seed and camera ray of pixel ``i`` depend
only on its global index (Raytracing.cl:170-184), so a frame is split by rows:
rank ``r`` of ``world`` renders the rows ``r, r+world, r+2*world, ...`` (row
interleaving balances sky rows against geometry rows) into a packed tile on its
own GPU, and rank 0 gathers the tiles with ONE collective over RCCL (xGMI) and
de-interleaves them.  The assembled frame is bit-identical to a one-GPU render.

The tile renderer is pluggable (``render_tile``), so the orchestration can be
exercised on CPU with the gloo backend and the oracle as the renderer.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

try:
    import torch
    import torch.distributed as dist
except ImportError:  # pragma: no cover
    torch = None
    dist = None


def tile_rows(npix: int, width: int, row0: int, row_step: int) -> int:
    """Rows of the frame (row width ``width``, ``npix`` pixels) in the tile ``row0::row_step``."""
    if npix <= 0 or width <= 0 or row0 < 0 or row_step <= 0:
        return 0
    H = (npix + width - 1) // width
    return 0 if row0 >= H else (H - row0 + row_step - 1) // row_step


def max_tile_rows(npix: int, width: int, world: int) -> int:
    return tile_rows(npix, width, 0, world)


def assemble(tiles, width: int, npix: int, world: int, out=None):
    """De-interleave ``world`` packed tiles (each padded to the largest tile) into one frame.

    Works on numpy arrays and torch tensors; returns ``[3*npix]``.
    """
    H = (npix + width - 1) // width
    mrows = max_tile_rows(npix, width, world)
    if torch is not None and isinstance(tiles[0], torch.Tensor):
        stack = torch.stack([t.reshape(mrows, width * 3) for t in tiles], 0)      # [world, mrows, W*3]
        frame = stack.transpose(0, 1).reshape(mrows * world, width * 3)[:H]      # row r = (r // world, r % world)
        flat = frame.reshape(-1)[: 3 * npix]
        if out is not None:
            out.copy_(flat)
            return out
        return flat.contiguous()
    stack = np.stack([np.asarray(t).reshape(mrows, width * 3) for t in tiles], 0)
    frame = stack.transpose(1, 0, 2).reshape(mrows * world, width * 3)[:H]
    flat = frame.reshape(-1)[: 3 * npix]
    if out is not None:
        out[:] = flat
        return out
    return np.ascontiguousarray(flat)


def render_distributed(render_tile: Callable, npix: int, width: int, rank: int, world: int, device=None,
                       group=None, gather: bool = True, quantize: Optional[Callable] = None):
    """Render this rank's rows with ``render_tile(row0, row_step, out_tile)`` and gather on rank 0.

    ``out_tile`` is a zero-initialised float32 tensor of ``3*width*max_rows``
    elements on ``device`` (the tail beyond this rank's rows stays zero).
    Returns the full frame (a flat tensor of ``3*npix``) on rank 0, the
    local tile on the other ranks.

    ``quantize(tile) -> uint8 tile`` (the output stage, e.g. ``gpu_rgb8``) runs on every rank
    before the gather, so the collective moves 1 byte per channel instead of 4.
    """
    mrows = max_tile_rows(npix, width, world)
    tile = torch.zeros(3 * width * mrows, dtype=torch.float32, device=device)
    render_tile(rank, world, tile)
    if quantize is not None:
        tile = quantize(tile)
    if world == 1:
        return tile[: 3 * npix]
    if not gather:
        return tile
    if rank == 0:
        bufs = [torch.empty_like(tile) for _ in range(world)]
        dist.gather(tile, gather_list=bufs, dst=0, group=group)
        return assemble(bufs, width, npix, world)
    dist.gather(tile, gather_list=None, dst=0, group=group)
    return tile


def gpu_tile_renderer(ctx, cam, env, npix: int, spp: int, max_bounce: int, device_index: int = 0,
                      stream: Optional[int] = None):
    """``render_tile`` backed by the HIP kernels (``rt_render_device``) on torch's current stream."""
    def render_tile(row0: int, row_step: int, out_tile):
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        ctx.render_device(cam, env, npix, spp, max_bounce, row0, row_step, out_tile.data_ptr(), s,
                          device_index=device_index)
    return render_tile


def gpu_rgb8(ctx, gamma: bool = False, device_index: int = 0, stream: Optional[int] = None):
    """``quantize`` for ``render_distributed``: the device output stage (``rt_rgb8_device``,
    FileManager.saveImg's ``(data*255).astype('uint8')``, gamma first if asked)."""
    def quantize(tile):
        out = torch.empty(tile.numel(), dtype=torch.uint8, device=tile.device)
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        ctx.rgb8_device(tile.data_ptr(), out.data_ptr(), tile.numel(), gamma, s, device_index=device_index)
        return out
    return quantize
