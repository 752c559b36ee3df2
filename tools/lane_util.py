"""Lane utilisation of the render loop from the instrumented launch (rt_count_work_detail): rays traced per
lane-iteration of the render loop (wave_outer x 64) and per lane-step of the traversal (wave_trav x 64).

    python tools/lane_util.py CONFIG [N ...]      (N: rank 0's tile of an N-GPU run; default 1)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from ensem3a_openclraytracer_amd import _native
    from ensem3a_openclraytracer_amd import workloads as W
    cfg = sys.argv[1]
    ns = [int(x) for x in sys.argv[2:]] or [1]
    sc, cam, env, npix, spp, mb, ibl = W.CONFIGS[cfg].inputs()
    ctx = _native.Context(device_ids=[0])
    ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
    ctx.set_env(ibl)
    for n in ns:
        c = ctx.count_work_detail(cam, env, npix, spp, mb, 0, n)
        lane_iters = 64 * c["wave_render_iters"]
        print(json.dumps({"config": cfg, "tile": n, **c,
                          "rays_per_lane_iteration": round(c["rays"] / max(1, lane_iters), 4),
                          "samples_per_ray": round(c["samples"] / max(1, c["rays"]), 4)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
