"""A/B of tree-walk variant libraries on C3/C4 (GPU box): bit-identity vs the default library at
4 spp, then full-config timing.   python tools/_ab_walk.py NAME:block[,NAME:block...]"""
import json, os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "ensem3a_openclraytracer_amd", "lib", "variants")
if len(sys.argv) > 2 and sys.argv[1] == "--one":
    sys.path.insert(0, ROOT)
    import numpy as np, torch
    from ensem3a_openclraytracer_amd import _native, workloads as W
    name, block, cfgs = sys.argv[2], int(sys.argv[3]), sys.argv[4].split(",")
    for cfg in cfgs:
        sc, cam, env, npix, spp, mb, ibl = W.CONFIGS[cfg].inputs()
        ctx = _native.Context(device_ids=[0])
        if block: ctx.set_option("block", block)
        for kv in filter(None, name.partition("@")[2].split("+")):   # NAME@key=value+key=value: options
            k, v = kv.split("=")
            ctx.set_option(k, int(v))
        ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
        ctx.set_env(ibl)
        info = ctx.scene_info()
        # AB_TILE=N: rank 0's tile of an N-GPU run (rows 0::N) instead of the whole frame; AB_REPS frames timed
        step = int(os.environ.get("AB_TILE", "1"))
        reps = int(os.environ.get("AB_REPS", "2"))
        width = int(cam[6])
        rows = (npix + width - 1) // width
        out = torch.empty(3 * width * ((rows + step - 1) // step), dtype=torch.float32, device="cuda")
        ctx.render_device(cam, env, npix, 4, mb, 0, step, out.data_ptr())
        torch.cuda.synchronize()
        small = out.cpu().numpy().copy()
        np.save(f"/tmp/ab_{cfg}_{step}_{name}.npy", small)
        ref = f"/tmp/ab_{cfg}_{step}_base.npy"
        same = bool(np.array_equal(np.load(ref), small)) if os.path.exists(ref) else None
        ctx.render_device(cam, env, npix, spp, mb, 0, step, out.data_ptr())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.render_device(cam, env, npix, spp, mb, 0, step, out.data_ptr())
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(json.dumps({"variant": name, "block": block, "cfg": cfg, "tile": step,
                          "Msamples/s": round(npix * spp / step / dt / 1e6, 1),
                          "ms": round(dt * 1e3, 3), "identical_4spp": same, "info": info}), flush=True)
        ctx.close()
else:
    for spec in sys.argv[1].split(","):
        name, block = spec.split(":")
        env = dict(os.environ)
        lib = name.split("@")[0]   # NAME@key=value+...: the library NAME with these rt_set_option values
        if lib != "base":
            env["ENSEM3A_RT_LIB"] = os.path.join(VDIR, f"lib{lib}.so")
        r = subprocess.run([sys.executable, __file__, "--one", name, block, os.environ.get("AB_CFGS", "C3,C4")],
                           env=env, timeout=600)
        if r.returncode != 0:
            print("FAILED", name, r.returncode, flush=True)
            sys.exit(1)
