"""Multi-rank orchestration (row-interleaved tiles + one gather) on CPU with gloo.

The per-rank tile renderer is the CPU oracle here (no GPU); on the GPU box the
same code path runs with the HIP renderer and the RCCL backend (bench.py).  The
assembled frame must be bit-identical to a single-rank render."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle.oracle as O
from ensem3a_openclraytracer_amd import distributed as D
from ensem3a_openclraytracer_amd import workloads as W


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("npix,width,world", [(12, 4, 2), (10, 4, 2), (10, 4, 3), (64 * 63, 64, 4), (7, 7, 2)])
def test_assemble_numpy_and_torch(npix, width, world):
    frame = np.arange(3 * npix, dtype=np.float32)
    H = (npix + width - 1) // width
    mrows = D.max_tile_rows(npix, width, world)
    tiles = []
    for r in range(world):
        t = np.zeros(3 * width * mrows, np.float32)
        rows = list(range(r, H, world))
        for k, row in enumerate(rows):
            n = min(width, npix - row * width)
            t[3 * width * k: 3 * width * k + 3 * n] = frame[3 * width * row: 3 * width * row + 3 * n]
        tiles.append(t)
    np.testing.assert_array_equal(D.assemble(tiles, width, npix, world), frame)
    got = D.assemble([torch.from_numpy(t) for t in tiles], width, npix, world)
    np.testing.assert_array_equal(got.numpy(), frame)


def _worker(rank, world, port, case, q, quantize=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wl = W.PARITY_CASES[case]
    sc, cam, env, npix, spp, mb, ibl = wl.inputs()
    osc = O.OracleScene.from_scene(sc, ibl)
    W_ = int(cam[6])

    def render_tile(row0, row_step, out_tile):
        t = O.render(osc, cam, env, npix, spp, mb, row0=row0, row_step=row_step, nthreads=2)
        out_tile[: t.size] = torch.from_numpy(t)

    qz = (lambda t: torch.from_numpy(O.rgb8(t.numpy()))) if quantize else None
    frame = D.render_distributed(render_tile, npix, W_, rank, world, quantize=qz)
    if rank == 0:
        q.put(frame.numpy().copy())
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world", [("cornell_64_s4", 2), ("serre_96x54_s4", 2), ("proto_64_s4", 3)])
def test_gloo_tiled_render_is_bit_identical(case, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    wl = W.PARITY_CASES[case]
    sc, cam, env, npix, spp, mb, ibl = wl.inputs()
    full = O.render(O.OracleScene.from_scene(sc, ibl), cam, env, npix, spp, mb, nthreads=4)
    np.testing.assert_array_equal(frame, full)


def test_gloo_quantized_gather_is_the_output_stage_of_the_full_frame():
    """Tiles quantized to 8 bits before the gather (4x fewer bytes on the wire) assemble into
    saveImg's (frame*255).astype(uint8) of the 1-rank frame."""
    case, world = "cornell_64_s4", 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    sc, cam, env, npix, spp, mb, ibl = W.PARITY_CASES[case].inputs()
    full = O.render(O.OracleScene.from_scene(sc, ibl), cam, env, npix, spp, mb, nthreads=4)
    assert frame.dtype == np.uint8
    np.testing.assert_array_equal(frame, O.rgb8(full))
