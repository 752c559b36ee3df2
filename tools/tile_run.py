"""Render rank 0's row tile (rows 0::N) of a BASELINE config a few times on device 0 -- the program a
rocprofv3 pass (tools/gpu_session.py ktpy= / pmcpy=) profiles for the N-GPU tile's counters.

    python tools/tile_run.py CONFIG N [FRAMES] [KEY=VALUE ...]   (rt_set_option values)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from ensem3a_openclraytracer_amd import _native
    from ensem3a_openclraytracer_amd import distributed as D
    from ensem3a_openclraytracer_amd import workloads as W
    cfg, n = sys.argv[1], int(sys.argv[2])
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    sc, cam, env, npix, spp, mb, ibl = W.CONFIGS[cfg].inputs()
    ctx = _native.Context(device_ids=[0])
    for kv in sys.argv[4:]:
        k, v = kv.split("=")
        ctx.set_option(k, int(v))
    ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
    ctx.set_env(ibl)
    width = int(cam[6])
    out = torch.empty(3 * width * D.tile_rows(npix, width, 0, n), dtype=torch.float32, device="cuda")
    for _ in range(frames):
        ctx.render_device(cam, env, npix, spp, mb, 0, n, out.data_ptr())
    torch.cuda.synchronize()
    ctx.close()
    print(f"tile_run {cfg} rows 0::{n}: {frames} frames", flush=True)


if __name__ == "__main__":
    main()
