"""Time one integer option of the native library over values, per config (GPU), plus parity.

    python tools/sweep_option.py OPTION v1,v2,... CONFIG [CONFIG ...] [--parity CASE,CASE]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("option")
    ap.add_argument("values")
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--parity", default="")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from ensem3a_openclraytracer_amd import _native
    from ensem3a_openclraytracer_amd import workloads as W
    vals = [int(v) for v in a.values.split(",")]
    if a.parity:
        import oracle.oracle as O
        from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher
        kl = KernelLauncher()
        for v in vals:
            kl.native.set_option(a.option, v)
            res = {}
            for case in a.parity.split(","):
                sc, cam, env, npix, spp, mb, ibl = W.PARITY_CASES[case].inputs()
                got = np.zeros(3 * npix, np.float32)
                kl.launch_Raytracing(got, sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData,
                                     sc.BVH.exportArray, cam, env, npix, spp, mb, ibl)
                ora = O.render(O.OracleScene.from_scene(sc, ibl), cam, env, npix, spp, mb, nthreads=16)
                res[case] = float(np.mean(got == ora))
            print(json.dumps({"parity": a.option, "value": v, "identical_frac": res}), flush=True)

    for name in a.configs:
        wl = W.CONFIGS[name]
        sc, cam, env, npix, spp, mb, ibl = wl.inputs()
        ctx = _native.Context(device_ids=[0])
        ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
        ctx.set_env(ibl)
        out = torch.empty(3 * npix, dtype=torch.float32, device="cuda")
        ref = None
        for v in vals:
            ctx.set_option(a.option, v)
            ctx.render_device(cam, env, npix, spp, mb, 0, 1, out.data_ptr())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                ctx.render_device(cam, env, npix, spp, mb, 0, 1, out.data_ptr())
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.reps
            img = out.cpu().numpy()
            same = None if ref is None else bool(np.array_equal(img, ref))
            ref = img if ref is None else ref
            print(json.dumps({"config": name, a.option: v, "ms": round(dt * 1e3, 3),
                              "Msamples_s": round(npix * spp / dt / 1e6, 1), "identical_to_first": same}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
