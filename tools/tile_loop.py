"""Render one row tile (rows 0::N of C2) a few times: a small driver for rocprofv3 counter passes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, ROOT)
import torch
from ensem3a_openclraytracer_amd import _native, distributed as D, workloads as W
n = int(sys.argv[1]); reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
opts = dict(kv.split("=") for kv in filter(None, (sys.argv[3] if len(sys.argv) > 3 else "").split(",")))
sc, cam, env, npix, spp, mb, ibl = W.CONFIGS["C2"].inputs()
ctx = _native.Context(device_ids=[0])
ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
ctx.set_env(ibl)
for k, v in opts.items(): ctx.set_option(k, int(v))
width = int(cam[6]); rows = D.max_tile_rows(npix, width, n)
out = torch.empty(3 * width * rows, dtype=torch.float32, device="cuda")
for _ in range(reps):
    ctx.render_device(cam, env, npix, spp, mb, 0, n, out.data_ptr())
torch.cuda.synchronize()
print("done", flush=True)
