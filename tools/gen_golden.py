"""Generate the golden fixtures from the REFERENCE kernel itself.

Runs on the GPU box: the reference's Kernels/Raytracing.cl, compiled from its own
sources by `make -C oracle ref` (in the container that has /root/reference) into
oracle/_ref/raytracing_gfx950.co, is executed by the ROCm OpenCL runtime through
oracle/refcl.py exactly as KernelLauncher.launch_Raytracing would enqueue it.
Known-answer tests call the reference's device functions through oracle/ref_cl/kat.cl.

    python tools/gen_golden.py OUTDIR      (then copy OUTDIR/*.npz to tests/golden/)

Outputs: ref_<case>.npz per parity case (inputs spec + reference image + kernel ms),
kat_reference.npz (inputs and outputs of every KAT), ref_timing.json (reference
kernel time at the benchmark configs on this GPU).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import refcl  # noqa: E402
from ensem3a_openclraytracer_amd import workloads as W  # noqa: E402


def render_ref(wl):
    sc, cam, env, npix, spp, mb, ibl = wl.inputs()
    out, ms = refcl.render(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.lightData, sc.materialData,
                           sc.BVH.exportArray, cam, env, npix, spp, mb, ibl)
    return out, ms, cam, env


def kat_inputs(rng):
    k = {}
    # rand: kernel seeds (i, 0) passed in naiveGI order (seed1, seed0) -> (0, i), plus random states
    s = np.concatenate([np.stack([np.zeros(256, np.uint32), np.arange(256, dtype=np.uint32)], 1),
                        rng.integers(0, 2**32, size=(256, 2), dtype=np.uint64).astype(np.uint32)])
    k["rand_seeds"] = s
    # camera: three cameras x pixel indices
    cams = []
    for (x, y, z, rx, ry, rz, w, h, dof) in [(0, -3.5, 0, 0, 0, 0, 4, 4, 45), (0, -3.5, 0, 0, 0, 0, 64, 64, 45),
                                             (7, -10, 10, -45, 0, 20, 96, 54, 75), (3, -10, 3, -5, 0, 15, 33, 17, 30)]:
        cams.append(np.array([x, y, z, rx, ry, rz, w, h, 1, dof * (3.14 / 180)], dtype=np.float64).astype(np.float32))
    k["cams"] = np.stack(cams)
    k["cam_idx"] = np.concatenate([np.arange(16), rng.integers(0, 4096, 200)]).astype(np.int32)
    # rotate: angle, axis, vector
    rot = rng.normal(size=(2000, 7)).astype(np.float32)
    rot[:, 0] = rng.uniform(-7, 7, 2000)
    rot[:8, 1:4] = [[1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 1], [0, 0, -1]]
    k["rotate_in"] = rot
    # intersect: random triangles + rays aimed near them
    n = 4000
    tri = rng.normal(size=(n, 9)).astype(np.float32)
    o = rng.normal(size=(n, 3)).astype(np.float32) * 3
    bary = rng.uniform(-0.2, 1.2, size=(n, 2))
    target = (tri[:, 0:3] + bary[:, :1] * (tri[:, 3:6] - tri[:, 0:3]) + bary[:, 1:] * (tri[:, 6:9] - tri[:, 0:3]))
    d = (target - o).astype(np.float32)
    d[:100] = d[:100] / np.linalg.norm(d[:100], axis=1, keepdims=True)
    k["intersect_in"] = np.concatenate([tri, d, o], 1).astype(np.float32)
    # box: rays vs boxes incl. zero direction components and flat boxes
    n = 4000
    r = rng.normal(size=(n, 6)).astype(np.float32)
    r[:400, 0] = 0.0
    r[400:800, 1] = 0.0
    r[800:900, 0:2] = 0.0
    lo = rng.normal(size=(n, 3)).astype(np.float32)
    hi = lo + np.abs(rng.normal(size=(n, 3))).astype(np.float32)
    hi[:300, 1] = lo[:300, 1]
    r[900:1000, 3] = lo[900:1000, 0]
    k["box_in"] = np.concatenate([r, lo, hi], 1).astype(np.float32)
    # ggx: material row + v, l, n
    n = 2000
    g = np.zeros((n, 15), np.float32)
    g[:, 0] = 2
    g[:, 1:4] = rng.uniform(0, 1, (n, 3))
    g[:, 4] = rng.uniform(0, 1, n)
    vv = rng.normal(size=(n, 9))
    for c in range(3):
        vv[:, 3 * c:3 * c + 3] /= np.linalg.norm(vv[:, 3 * c:3 * c + 3], axis=1, keepdims=True)
    g[:, 6:15] = vv
    k["ggx_in"] = g
    # ibl / texel
    dirs = rng.normal(size=(4000, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    dirs[:6] = [[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]]
    k["ibl_dirs"] = dirs.astype(np.float32)
    k["small_ibl"] = rng.integers(0, 256, size=(5, 7, 4), dtype=np.uint8)
    xs, ys = np.meshgrid(np.arange(-2, 10), np.arange(-2, 8), indexing="ij")
    k["texel_xy"] = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    # hemisphere samplers
    nn = rng.normal(size=(3000, 3))
    nn /= np.linalg.norm(nn, axis=1, keepdims=True)
    nn[:4] = [[0, 0, 1], [0, 0, -1], [0.0, 0.9626, 0.2708], [-0.9626, -0.2708, 0]]
    k["hemi_n"] = nn.astype(np.float32)
    k["hemi_seeds_in"] = rng.integers(0, 2**32, size=(3000, 2), dtype=np.uint64).astype(np.uint32)
    # elementary functions
    k["math_x"] = np.concatenate([rng.uniform(-10, 10, 4000), rng.uniform(-1, 1, 4000)]).astype(np.float32)
    k["math_y"] = rng.uniform(-10, 10, 8000).astype(np.float32)
    return k


def trace_rays(sc, rng, n=3000):
    """Rays from the Cornell camera region and from random points, random directions."""
    o = rng.normal(size=(n, 3)) * 0.6
    o[: n // 2] = [0, -3.5, 0]
    d = rng.normal(size=(n, 3))
    d[: n // 2, 1] = np.abs(d[: n // 2, 1]) + 1.0
    return np.concatenate([d, o], 1).astype(np.float32)


def main(outdir):
    os.makedirs(outdir, exist_ok=True)
    assert refcl.available(), "oracle/_ref is not built (make -C oracle ref where the reference exists)"
    refcl.open_program(refcl.RT_CO)
    dev = refcl.device_name()
    print("OpenCL device:", dev, flush=True)
    meta = {"device": dev, "generator": "tools/gen_golden.py", "time": time.strftime("%Y-%m-%d %H:%M:%S")}
    meta["image_support"] = refcl.image_support()
    print("OpenCL image support:", meta["image_support"], flush=True)
    if meta["image_support"]:
        for name, wl in W.PARITY_CASES.items():
            t = time.time()
            out, ms, cam, env = render_ref(wl)
            np.savez_compressed(os.path.join(outdir, f"ref_{name}.npz"), out=out, cam=cam, env=env,
                                spec=np.frombuffer(json.dumps(dict(
                                    scene=wl.scene, width=wl.width, height=wl.height, spp=wl.spp,
                                    max_bounce=wl.max_bounce, ibl=wl.ibl, kernel_ms=ms, **meta)).encode(),
                                    np.uint8))
            print(f"{name}: {ms:.2f} ms kernel, {time.time() - t:.1f} s, mean {out.mean():.5f}", flush=True)

    rng = np.random.default_rng(1234)
    k = kat_inputs(rng)
    res = dict(k)
    res["rand_out"], res["rand_state"] = refcl.kat_rand(k["rand_seeds"], 8)
    res["cam_out"] = np.stack([refcl.kat_camera(c, k["cam_idx"]) for c in k["cams"]])
    res["rotate_out"] = refcl.kat_rotate(k["rotate_in"])
    res["intersect_out"] = refcl.kat_intersect(k["intersect_in"])
    res["box_out"] = refcl.kat_box(k["box_in"])
    res["ggx_out"] = refcl.kat_ggx(k["ggx_in"])
    prev = W.ibl_preview()
    res["sphmap_out"] = refcl.kat_sphmap(k["ibl_dirs"])
    if meta["image_support"]:
        res["ibl_out"] = refcl.kat_ibl(prev, k["ibl_dirs"])
        res["ibl_small_out"] = refcl.kat_ibl(k["small_ibl"], k["ibl_dirs"])
        res["texel_out"] = refcl.kat_texel(k["small_ibl"], k["texel_xy"])
    for kind in (1, 2):
        d, s = refcl.kat_hemi(kind, k["hemi_n"], k["hemi_seeds_in"].copy())
        res[f"hemi{kind}_out"], res[f"hemi{kind}_state"] = d, s
    for fn in range(8):
        res[f"math{fn}_out"] = refcl.kat_math(fn, k["math_x"], k["math_y"])
    for sname in ("cornell", "monkey", "serre", "proto"):
        sc = W.load_scene(sname)
        rays = trace_rays(sc, rng)
        res[f"trace_{sname}_rays"] = rays
        res[f"trace_{sname}_out"] = refcl.kat_trace(sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.BVH.exportArray, rays)
    res["meta"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(os.path.join(outdir, "kat_reference.npz"), **res)
    print("KATs written", flush=True)
    if not meta["image_support"]:
        with open(os.path.join(outdir, "ref_timing.json"), "w") as f:
            json.dump(dict(meta, note="reference Raytracing kernel needs image2d_t; no image support here"), f)
        return

    # reference kernel time at the benchmark configurations on this GPU
    timing = dict(meta)
    for key in ("C1", "C2"):
        wl = W.CONFIGS[key]
        out, ms, _, _ = render_ref(wl)
        timing[key] = dict(workload=wl.name, kernel_ms=ms, msamples_per_s=wl.samples / (ms * 1e-3) / 1e6,
                           channel_mean=[float(x) for x in out.reshape(-1, 3).mean(0)])
        print(key, timing[key], flush=True)
        if key == "C2":
            np.save(os.path.join(outdir, "ref_C2_full.npy"), out)
    with open(os.path.join(outdir, "ref_timing.json"), "w") as f:
        json.dump(timing, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/golden")
