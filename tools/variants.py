"""Build experimental variants of the native library and A/B them on the GPU box.

    python tools/variants.py build NAME=DEF1,DEF2 ...      (here: compiles build/variants/libNAME.so)
    python tools/variants.py run NAME ...                   (GPU box: parity + C2 timing per variant)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "ensem3a_openclraytracer_amd", "lib", "variants")  # travels to the GPU box (build/ does not)


def build(specs):
    sys.path.insert(0, ROOT)
    from ensem3a_openclraytracer_amd import _build
    for spec in specs:
        name, _, defs = spec.partition("=")
        defines = tuple(d for d in defs.split(",") if d)
        path = _build.build(defines=defines or ("RT_VARIANT_BASE=1",), out=os.path.join(VDIR, f"lib{name}.so"))
        print("built", path)


CHECK = r'''
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.environ["ROOT"])
from ensem3a_openclraytracer_amd import workloads as W
from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher
import oracle.oracle as O
from oracle import compare
kl = KernelLauncher(traversal=os.environ.get("TRAV", "fast"), bvh=os.environ.get("BVH", "sah"))
res = {}
for case in ["furnace_64_s4", "monkey_c3_64_s4", "serre_96x54_s4", "proto_64_s4", "cornell_128_s16"]:
    sc, cam, env, npix, spp, mb, ibl = W.PARITY_CASES[case].inputs()
    out = np.zeros(3 * npix, np.float32)
    kl.launch_Raytracing(out, sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData,
                         sc.BVH.exportArray, cam, env, npix, spp, mb, ibl)
    ora = O.render(O.OracleScene.from_scene(sc, ibl), cam, env, npix, spp, mb, nthreads=16)
    st = compare.stats(out, ora)
    res[case] = round(st["frac_identical"], 5)
print(json.dumps(res))
'''


def run(names):
    env = dict(os.environ, ROOT=ROOT)
    for name in names:
        env["ENSEM3A_RT_LIB"] = os.path.join(VDIR, f"lib{name}.so")
        r = subprocess.run([sys.executable, "-c", CHECK], env=env, capture_output=True, text=True, timeout=300)
        parity = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else "ERR " + r.stderr[-300:]
        perf = []
        for cfg in os.environ.get("VAR_CONFIGS", "C2").split(","):
            steps = "10" if cfg == "C2" else "2"
            b = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", steps, "--warmup", "1",
                                "--no-cpu-baseline", "--config", cfg, "--bvh", os.environ.get("BVH", "sah")],
                               env=env, capture_output=True, text=True, timeout=600)
            try:
                d = json.loads(b.stdout.strip().splitlines()[-1])
                perf.append(f'{cfg} {d["value"]:.1f} Msamples/s ({d["roofline"]["kernel_ms"]:.2f} ms)')
            except Exception:
                perf.append(f"{cfg} ERR " + b.stderr[-300:])
        perf = "; ".join(perf)
        print(f"{name}: {perf} | identical-vs-oracle {parity}", flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]](sys.argv[2:])
