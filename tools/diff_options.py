"""Render a parity case with two native option sets and against the CPU oracle; print where they differ.

    python tools/diff_options.py CASE "opt=v,..." ["opt=v,..."] [row0 row_step]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(spec):
    return {k: int(v) for k, v in (kv.split("=") for kv in filter(None, spec.split(",")))}


def main():
    import torch
    from ensem3a_openclraytracer_amd import _native
    from ensem3a_openclraytracer_amd import workloads as W
    import oracle.oracle as O
    wl = W.PARITY_CASES.get(sys.argv[1]) or W.CONFIGS[sys.argv[1]]
    a = parse(sys.argv[2]) if len(sys.argv) > 2 else {}
    b = parse(sys.argv[3]) if len(sys.argv) > 3 else {}
    row0 = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    step = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    sc, cam, env, npix, spp, mb, ibl = wl.inputs()
    ctx = _native.Context(device_ids=[0])
    ctx.set_scene(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.BVH.exportArray)
    ctx.set_env(ibl)
    width = int(cam[6])
    rows = _native.tile_rows(npix, width, row0, step)
    outs = []
    for o in (a, b):
        for k, v in o.items():
            ctx.set_option(k, v)
        t = torch.zeros(3 * width * rows, dtype=torch.float32, device="cuda")
        ctx.render_device(cam, env, npix, spp, mb, row0, step, t.data_ptr())
        torch.cuda.synchronize()
        outs.append(t.cpu().numpy())
    ref = O.render(O.OracleScene.from_scene(sc, ibl), cam, env, npix, spp, mb, row0=row0, row_step=step, nthreads=8)
    for name, x in (("a", outs[0]), ("b", outs[1])):
        d = np.nonzero(x.view(np.uint32) != ref.view(np.uint32))[0]
        px = np.unique(d // 3)
        print(json.dumps({"set": name, "opts": a if name == "a" else b, "diff_values": int(d.size),
                          "diff_pixels": int(px.size), "first": px[:12].tolist(),
                          "max_abs": float(np.abs(x - ref).max()) if d.size else 0.0}), flush=True)
        r3, x3 = ref.reshape(-1, 3), x.reshape(-1, 3)
        for q in px[:4]:
            same = np.nonzero((r3 == x3[q]).all(axis=1))[0]
            print(f"  pixel {q}: gpu {x3[q].tolist()} oracle {r3[q].tolist()} "
                  f"(oracle pixels with the gpu value: {same[:8].tolist()})", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
