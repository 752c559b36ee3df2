import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, ROOT)
from ensem3a_openclraytracer_amd import workloads as W
from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher
import oracle.oracle as O
np.set_printoptions(precision=9, linewidth=200, suppress=False)
kl = KernelLauncher(traversal="ref")
wl = W.Workload("dbg", "monkey", 32, 32, 1, max_bounce=1, overrides=((4, 3.0, (0.88, 1.0, 1.0), None),))
sc, cam, env, npix, spp, mb, ibl = wl.inputs()
osc = O.OracleScene.from_scene(sc, ibl)
kl.launch_Raytracing(np.zeros(3*npix, np.float32), sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData,
                     sc.BVH.exportArray, cam, env, npix, spp, mb, ibl)
for pix in (658,):
    lo, oo = O.pixel_log(osc, cam, env, npix, spp, mb, pix)
    lg, og = kl.native.debug_pixel_log(1, cam, env, npix, spp, mb, pix)
    print("pixel", pix, "oracle", oo, "gpu", og)
    print("oracle events\n", lo)
    print("gpu events\n", lg)
