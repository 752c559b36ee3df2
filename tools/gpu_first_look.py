"""First GPU look: HIP path vs CPU oracle vs reference fixtures, and C2 timing.

    python tools/gpu_first_look.py [golden_dir]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ensem3a_openclraytracer_amd import workloads as W  # noqa: E402
from ensem3a_openclraytracer_amd import _native  # noqa: E402
from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher  # noqa: E402
import oracle.oracle as O  # noqa: E402
from oracle import compare  # noqa: E402


def main(golden):
    kl = KernelLauncher()
    ctx = kl.native
    # numerics contract: device vs oracle bit-exact
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(-20, 20, 100000), rng.uniform(-1, 1, 100000)]).astype(np.float32)
    y = rng.uniform(-5, 5, x.size).astype(np.float32)
    for name, fn in O.MATH_FN.items():
        g = ctx.debug_math(fn, x, y)
        c = O.math(name, x, y)
        same = np.array_equal(g.view(np.uint32), c.view(np.uint32)) or np.array_equal(g, c, equal_nan=True)
        print(f"math {name}: bit-identical={same} mismatches={int((g != c).sum() - (np.isnan(g) & np.isnan(c)).sum())}",
              flush=True)
    res = {}
    for name, wl in W.PARITY_CASES.items():
        sc, cam, env, npix, spp, mb, ibl = wl.inputs()
        osc = O.OracleScene.from_scene(sc, ibl)
        ora = O.render(osc, cam, env, npix, spp, mb, nthreads=16)
        row = {}
        for trav in ("ref", "fast"):
            kl.set_traversal(trav)
            out = np.zeros(3 * npix, np.float32)
            kl.launch_Raytracing(out, sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData,
                                 sc.BVH.exportArray, cam, env, npix, spp, mb, ibl)
            st = compare.stats(out, ora)
            row[trav] = dict(vs_oracle_identical=st["frac_identical"], vs_oracle_within=st["frac_within"])
            gp = os.path.join(golden, f"ref_{name}.npz")
            if os.path.exists(gp):
                ref = np.load(gp)["out"]
                st2 = compare.stats(out, ref)
                row[trav]["vs_reference"] = st2
        if os.path.exists(os.path.join(golden, f"ref_{name}.npz")):
            row["oracle_vs_reference"] = compare.stats(ora, np.load(os.path.join(golden, f"ref_{name}.npz"))["out"])
        res[name] = row
        print(name, json.dumps(row), flush=True)
    # C2 timing
    wl = W.CONFIGS["C2"]
    sc, cam, env, npix, spp, mb, ibl = wl.inputs()
    for trav in ("fast", "ref"):
        kl.set_traversal(trav)
        out = np.zeros(3 * npix, np.float32)
        args = (out, sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData, sc.BVH.exportArray,
                cam, env, npix, spp, mb, ibl)
        kl.launch_Raytracing(*args)
        ts = []
        for _ in range(3):
            t = time.time()
            kl.launch_Raytracing(*args)
            ts.append(time.time() - t)
        t = min(ts)
        print(f"C2 {trav}: {t * 1e3:.1f} ms  {wl.samples / t / 1e6:.1f} Msamples/s (host-inclusive)", flush=True)
        refp = os.path.join(golden, "ref_C2_full.npy")
        if os.path.exists(refp):
            print("  vs reference C2:", json.dumps(compare.stats(out, np.load(refp))), flush=True)
        cnt = ctx.count_work(cam, env, npix, spp, mb)
        print("  counts per sample:", {k: v / wl.samples for k, v in cnt.items()}, flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/golden")
