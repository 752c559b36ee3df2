import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, ROOT)
from ensem3a_openclraytracer_amd import workloads as W
from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher
import oracle.oracle as O
from oracle import compare
kl = KernelLauncher(traversal="ref")
base = W.PARITY_CASES["monkey_c3_64_s4"]
variants = {
  "c3": base.overrides,
  "glass_only": ((4, 3.0, (0.88, 1.0, 1.0), None),),
  "glossy_only": ((0, 2.0, None, 0.2),),
}
for vname, ov in variants.items():
  for (spp, mb) in [(1, 0), (1, 1), (1, 4), (4, 0), (4, 4)]:
    for env_override in (None, "nosun", "noibl"):
      wl = W.Workload("dbg", "monkey", 32, 32, spp, max_bounce=mb, overrides=ov)
      sc, cam, env, npix, spp_, mb_, ibl = wl.inputs()
      env = env.copy()
      if env_override == "nosun": env[3] = 0
      if env_override == "noibl": env[4] = 0
      osc = O.OracleScene.from_scene(sc, ibl)
      ora = O.render(osc, cam, env, npix, spp, mb, nthreads=8)
      out = np.zeros(3 * npix, np.float32)
      kl.launch_Raytracing(out, sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData,
                           sc.BVH.exportArray, cam, env, npix, spp, mb, ibl)
      st = compare.stats(out, ora)
      bad = np.nonzero((out.reshape(-1,3) != ora.reshape(-1,3)).any(1))[0]
      print(vname, spp, mb, env_override, "identical", round(st["frac_identical"], 4), "first bad", bad[:5].tolist(),
            (out.reshape(-1,3)[bad[:2]].tolist(), ora.reshape(-1,3)[bad[:2]].tolist()) if len(bad) else "", flush=True)
