"""SIMD efficiency of the render loop (GPU): lane work vs wave-level iterations.

    python tools/wave_stats.py [CONFIG ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensem3a_openclraytracer_amd import _native  # noqa: E402
from ensem3a_openclraytracer_amd import workloads as W  # noqa: E402

for name in sys.argv[1:] or ["C2"]:
    wl = W.CONFIGS[name] if name in W.CONFIGS else W.PARITY_CASES[name]
    scene, cam, env, npix, spp, mb, ibl = wl.inputs()
    for bvh in (_native.RT_BVH_SAH, _native.RT_BVH_REFERENCE):
        ctx = _native.Context(device_ids=[0])
        ctx.set_option("bvh", bvh)
        ctx.set_scene(scene.V_p, scene.V_n, scene.V_uv, scene.faceData, scene.materialData, scene.BVH.exportArray)
        ctx.set_env(ibl)
        c = ctx.wave_counts(cam, env, npix, spp, mb)
        samples = npix * spp
        lane_iters = c["node_fetches"] + c["tri_tests"]
        out = {"config": name, "bvh": "sah" if bvh == _native.RT_BVH_SAH else "reference",
               "per_sample": {k: round(v / samples, 3) for k, v in c.items()},
               "trav_simd_eff": round(lane_iters / max(1, 64 * c["wave_trav_iters"]), 4),
               "trav_iters_per_wave_render_iter": round(c["wave_trav_iters"] / max(1, c["wave_render_iters"]), 2),
               "rays_per_lane_render_iter": round(c["rays"] / max(1, 64 * c["wave_render_iters"]), 4),
               "trav_cycle_share": round(c["cycles_trav"] / max(1, c["cycles_trav"] + c["cycles_shade"]), 4)}
        print(json.dumps(out), flush=True)
        ctx.close()
