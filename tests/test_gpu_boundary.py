"""GPU tests of the drop-in boundary's process / stream contract (include/rt_api.h).

* the single-GPU drop-in path (KernelLauncher) runs without torch, and a torch imported
  afterwards shares the HIP runtime the library loaded;
* launches of one context on different streams are ordered (they share the per-device
  pixel counters and launch constants), so overlapping them never corrupts a frame;
* scene re-uploads wait for launches still in flight on a caller's stream.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from ensem3a_openclraytracer_amd import _native
from ensem3a_openclraytracer_amd import workloads as W

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

NO_TORCH = r'''
import sys
sys.path.insert(0, sys.argv[1])
import numpy as np
from ensem3a_openclraytracer_amd import workloads as W
from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher
sc, cam, env, npix, spp, mb, ibl = W.PARITY_CASES["cornell_64_s4"].inputs()
kl = KernelLauncher(None, None, 0, None)
out = np.zeros(3 * npix, np.float32)
kl.launch_Raytracing(out, sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData,
                     sc.BVH.exportArray, cam, env, npix, spp, mb, ibl)
assert "torch" not in sys.modules, "the drop-in path imported torch"
import torch
d = torch.empty(3 * npix, dtype=torch.float32, device="cuda")
s = torch.cuda.Stream()
kl.native.render_device(cam, env, npix, spp, mb, 0, 1, d.data_ptr(), s.cuda_stream)
s.synchronize()
assert np.array_equal(d.cpu().numpy(), out), "torch-stream render differs"
kl.close()
print("ok")
'''


def test_library_loads_without_torch_and_shares_the_runtime():
    r = subprocess.run([sys.executable, "-c", NO_TORCH, ROOT], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]


def _ctx(case, size=None):
    wl = W.PARITY_CASES[case]
    if size:
        wl = wl.with_size(*size)
    sc, cam, env, npix, spp, mb, ibl = wl.inputs()
    ctx = _native.Context(device_ids=[0])
    ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
    ctx.set_env(ibl)
    return ctx, cam, env, npix, spp, mb


@pytest.mark.parametrize("case", ["cornell_128_s16", "monkey_c3_64_s4"])
def test_launches_on_two_streams_do_not_race(case):
    import torch
    ctx, cam, env, npix, spp, mb = _ctx(case)
    cam2 = cam.copy()
    cam2[3] += 7.0   # another camera rotation: another per-launch constant block
    want1 = ctx.render(cam, env, npix, spp, mb)
    want2 = ctx.render(cam2, env, npix, 2 * spp, mb)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.empty(3 * npix, dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    for _ in range(3):
        a.fill_(-1.0)
        b.fill_(-1.0)
        torch.cuda.synchronize()
        ctx.render_device(cam, env, npix, spp, mb, 0, 1, a.data_ptr(), s1.cuda_stream)
        ctx.render_device(cam2, env, npix, 2 * spp, mb, 0, 1, b.data_ptr(), s2.cuda_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(a.cpu().numpy(), want1)
        np.testing.assert_array_equal(b.cpu().numpy(), want2)
    ctx.close()


@pytest.mark.parametrize("first,second,size", [
    ("monkey_c3_64_s4", "cornell_64_s4", (512, 512, 64)),     # smaller scene: buffers reused
    ("cornell_64_s4", "monkey_c3_64_s4", (1024, 1024, 256)),  # larger scene: buffers freed + reallocated
])
def test_scene_upload_waits_for_a_launch_in_flight(first, second, size):
    """rt_set_scene right after an asynchronous launch on a caller's stream: the launch still
    renders the old scene (the upload, and any free of a buffer it reads, is ordered after it)."""
    import torch
    ctx, cam, env, npix, spp, mb = _ctx(first, size)   # ~10-30 ms in flight
    want = ctx.render(cam, env, npix, spp, mb)
    sc2, *_ = W.PARITY_CASES[second].inputs()
    s = torch.cuda.Stream()
    a = torch.empty(3 * npix, dtype=torch.float32, device="cuda")
    ctx.render_device(cam, env, npix, spp, mb, 0, 1, a.data_ptr(), s.cuda_stream)
    ctx.set_scene(sc2.V_p, sc2.V_n, sc2.V_uv, sc2.faceData, sc2.materialData, sc2.BVH.exportArray)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.cpu().numpy(), want)
    ctx.close()


@pytest.mark.parametrize("slots", [2, 3])
@pytest.mark.parametrize("case", ["cornell_128_s16", "monkey_c3_64_s4", "serre_96x54_s4"])
def test_multi_device_launcher_deinterleaves_rows(case, slots):
    """KernelLauncher(device=[0, 0, ...]): the single-process multi-device path of the Tk UI.  rt_render
    launches every device slot on its interleaved rows (row r on slot r mod n, each slot with its own
    stream and buffers -- here all on GPU 0), copies each tile back and de-interleaves the rows into the
    caller's array (rt_api.hip render_host).  The frame, float32 and fused rgb8, is the one-device
    frame bit for bit, including a partial last row."""
    from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher
    sc, cam, env, npix, spp, mb, ibl = W.PARITY_CASES[case].inputs()
    one = KernelLauncher(None, None, 0, None)
    multi = KernelLauncher(None, None, [0] * slots, None)
    try:
        assert multi.native.n_devices == slots
        for n in (npix, npix - int(cam[6]) // 2 - 1):
            args = (sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData, sc.BVH.exportArray,
                    cam, env, n, spp, mb, ibl)
            want = np.zeros(3 * n, np.float32)
            one.launch_Raytracing(want, *args)
            got = np.full(3 * n, -1.0, np.float32)
            multi.launch_Raytracing(got, *args)
            np.testing.assert_array_equal(got, want)
            want8 = np.zeros(3 * n, np.uint8)
            one.launch_Raytracing_rgb8(want8, *args, gamma=True)
            got8 = np.zeros(3 * n, np.uint8)
            multi.launch_Raytracing_rgb8(got8, *args, gamma=True)
            np.testing.assert_array_equal(got8, want8)
    finally:
        one.close()
        multi.close()


RCCL_ONE_RANK = r'''
import os, sys
sys.path.insert(0, sys.argv[1])
import numpy as np
import torch
import torch.distributed as dist
from ensem3a_openclraytracer_amd import _native
from ensem3a_openclraytracer_amd import distributed as D
from ensem3a_openclraytracer_amd import workloads as W
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2], RANK="0", WORLD_SIZE="1")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
assert dist.get_backend() == "nccl"
sc, cam, env, npix, spp, mb, ibl = W.PARITY_CASES["monkey_c3_64_s4"].inputs()
ctx = _native.Context(device_ids=[0])
ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
ctx.set_env(ibl)
w = int(cam[6])
tile = D.render_distributed(D.gpu_tile_renderer(ctx, cam, env, npix, spp, mb), npix, w, 0, 1, device="cuda",
                            gather=False)
bufs = [torch.empty_like(tile)]
dist.gather(tile, gather_list=bufs, dst=0)   # RCCL
frame = D.assemble(bufs, w, npix, 1)
torch.cuda.synchronize()
want = ctx.render(cam, env, npix, spp, mb)
assert np.array_equal(frame.cpu().numpy(), want), "RCCL-gathered frame differs"
ctx.close()
dist.destroy_process_group()
print("rccl ok")
'''


def test_rccl_gather_path_on_the_device():
    """The multi-GPU path's collective on hardware: torch.distributed over RCCL ('nccl') with one rank,
    the HIP tile renderer and the gather of distributed.render_distributed -- the frame equals the
    direct render.  (Two ranks cannot share one GPU under RCCL; the 8-GPU run is the driver's.)"""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", RCCL_ONE_RANK, ROOT, str(port)], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0 and "rccl ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
