"""Time the tile one rank of an N-GPU run renders (rows 0::N) under sets of native options
(rt_set_option), each checked bit-identical against the first set.  Separates latency exposure
(few resident waves: option "waves") from the one-pixel-per-lane regime of small tiles (option
"team").

    python tools/occupancy_probe.py CONFIG N,N,... "opt=v,opt=v;opt=v;..."
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULTS = {"spec": -1, "slices": -1, "team": 0, "sun_cache": 1, "walk_team": 0, "brute_max": 64, "waves": 0, "block": 128, "fixed_point": 1, "pilot": -1, "pilot_chunk": 0, "pilot_levels": 0, "stack_lds": 0, "step": 0, "resume_min": -1, "bvh_width": 0}


def main():
    import torch
    from ensem3a_openclraytracer_amd import _native
    from ensem3a_openclraytracer_amd import distributed as D
    from ensem3a_openclraytracer_amd import workloads as W
    name = sys.argv[1] if len(sys.argv) > 1 else "C2"
    ns = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,8").split(",")]
    sets = []
    for spec in (sys.argv[3] if len(sys.argv) > 3 else "team=1;team=0").split(";"):
        o = dict(DEFAULTS)
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            o[k.strip()] = int(v)
        sets.append(o)
    sc, cam, env, npix, spp, mb, ibl = W.CONFIGS[name].inputs()
    ctx = _native.Context(device_ids=[0])
    ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
    ctx.set_env(ibl)
    width = int(cam[6])
    for n in ns:
        rows = D.max_tile_rows(npix, width, n)
        out = torch.empty(3 * width * rows, dtype=torch.float32, device="cuda")
        ref = None
        for o in sets:
            for k, v in o.items():
                ctx.set_option(k, v)
            ctx.render_device(cam, env, npix, spp, mb, 0, n, out.data_ptr())
            torch.cuda.synchronize()
            same = True
            if ref is None:
                ref = out.clone()
            else:
                same = bool(torch.equal(ref, out))
            reps = 3 if n == 1 else 5
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.render_device(cam, env, npix, spp, mb, 0, n, out.data_ptr())
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            print(json.dumps({"config": name, "n": n, "opts": {k: v for k, v in o.items() if v != DEFAULTS.get(k)},
                              "tile_ms": round(dt * 1e3, 3), "identical": same}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
