"""SIMD efficiency of the render loop (GPU): lane work vs wave-level iterations, per option set.

    python tools/wave_stats.py CONFIG[,CONFIG...] ["opt=v,opt=v;opt=v;..."] [OUT.jsonl]

Prints, per config and option set (rt_set_option), the instrumented kernel's counters per sample
and the derived loop efficiencies (rt_count_work_detail).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensem3a_openclraytracer_amd import _native  # noqa: E402
from ensem3a_openclraytracer_amd import workloads as W  # noqa: E402

# rt_set_option defaults of the options a set may change (rt_api.hip)
DEFAULTS = {"spec": -1, "slices": -1, "pilot": -1, "resume_min": -1, "handout": -1, "bvh_width": 0, "brute_max": 64,
            "block": 128, "fixed_point": 1, "sun_cache": 1}
names = (sys.argv[1] if len(sys.argv) > 1 else "C3").split(",")
sets = [dict(kv.split("=") for kv in filter(None, spec.split(",")))
        for spec in (sys.argv[2] if len(sys.argv) > 2 else "").split(";")]
for name in names:
    wl = W.CONFIGS[name] if name in W.CONFIGS else W.PARITY_CASES[name]
    scene, cam, env, npix, spp, mb, ibl = wl.inputs()
    ctx = _native.Context(device_ids=[0])
    ctx.set_scene(scene.V_p, scene.V_n, scene.V_uv, scene.faceData, scene.materialData, scene.BVH.exportArray)
    ctx.set_env(ibl)
    for opts in sets:
        for k, v in opts.items():
            ctx.set_option(k, int(v))
        c = ctx.count_work_detail(cam, env, npix, spp, mb)
        samples = max(1, c["samples"])
        lane_iters = c["node_fetches"] + c["tri_tests"]
        out = {"config": name, "opts": opts,
               "per_sample": {k: round(v / samples, 3) for k, v in c.items()},
               "trav_simd_eff": round(lane_iters / max(1, 64 * c["wave_trav_iters"]), 4),
               "trav_iters_per_wave_render_iter": round(c["wave_trav_iters"] / max(1, c["wave_render_iters"]), 2),
               "rays_per_lane_render_iter": round(c["rays"] / max(1, 64 * c["wave_render_iters"]), 4),
               "trav_cycle_share": round(c["cycles_trav"] / max(1, c["cycles_trav"] + c["cycles_shade"]), 4)}
        print(json.dumps(out), flush=True)
        if len(sys.argv) > 3:   # committed evidence (profiles/rNN_wave_stats.jsonl)
            with open(sys.argv[3], "a") as f:
                f.write(json.dumps(out) + "\n")
        for k in opts:   # back to the defaults for the next set
            ctx.set_option(k, DEFAULTS.get(k, 0))
    ctx.close()
