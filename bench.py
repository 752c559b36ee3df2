"""Benchmark of the path-tracing hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--traversal fast|ref] [--bvh sah|reference]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one full frame of the configuration (default C2: Cornell box
1024x1024, 64 spp, maxBounce 4): every rank renders its row-interleaved tile with
the HIP kernel (scene and IBL already resident in HBM), rank 0 gathers the tiles
over RCCL and assembles the frame (frame k's gather overlaps frame k+1's render:
two tile buffers; the timed region ends after the last frame is assembled).  K steps are timed between barrier +
synchronize fences; the max over ranks is reported.  value = W*H*spp / time in
Msamples/s (whole job; the frame size is fixed, so scaling is "strong").

Extra fields (DESIGN.md 5 derives every number):
  roofline      -- the render kernel against the bound of the path that ran:
                   * brute-force path (scenes of <= brute_max triangles: C1/C2):
                     bound "valu", achieved = algorithmic VALU lane-operations per
                     launch (VALU_OPS per unit x the unit counts of the SAME
                     traversal, rt_count_work_detail) / the kernel's average
                     duration from HIP events on its stream; peak = the FP32 vector
                     issue rate (256 CUs x 4 SIMD x 32 lanes x 2.4 GHz).
                   * tree walk (C3-C5): bound "cache", achieved = SURVEY 8(d)
                     algorithmic bytes per launch / kernel time, peak = the
                     L2 delivery rate incl. L1 reuse (36.9 TB/s, MI355X_MICROARCH.md):
                     the walk's bytes are served by the vL1D / L2, not HBM;
                     hbm_measured = PMC HBM bytes / kernel time vs 8 TB/s.
                   traffic = PMC-measured HBM bytes per launch (committed rocprofv3
                   summary in profiles/), issued = PMC-measured VALU lane slots
                   (SQ_INSTS_VALU x 64) per launch, when committed.
  host_boundary -- rt_render (launch_Raytracing's blocking C-ABI: kernel + copy of
                   the frame into caller memory), timed over the same W/K steps.
  configs       -- C1 (20 steps), C3 and C4 (5 steps) and C5 (2 steps), 1+ warmup, timed the same way (per-frame min / median
                   and the GPU clock beside them); at N=1 on one device (with their roofline and the CPU
                   oracle's rate: C1 whole frame, C3-C5 per sample at 16 spp), at N>1 through the same
                   row tiles + RCCL gather as the headline (every config's strong scaling).
  cold_call     -- per config line: a fresh KernelLauncher's first launch_Raytracing into host memory
                   (SURVEY 8(d)'s t_render: packing + uploads + IBL + render + read-back), split.
  cpu_baseline  -- the CPU oracle (a C restatement of the reference kernel, OpenMP)
                   timed on this host on a bounded row sample of the same frame.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/s Cornell box 1024x1024 64spp; 1/2/4/8-GPU scaling; HBM %peak"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
CACHE_PEAK_GBS = 36900.0       # L2 (all XCDs) delivery incl. L1 reuse, MI355X_MICROARCH.md "L2 (per XCD)"
VALU_PEAK_TOPS = 78.6432       # 256 CUs x 4 SIMD x 32 lanes/clk x 2.4 GHz: VALU lane-ops/s (157.3 TFLOPS FP32 = 2 x this, FMA)

# Algorithmic VALU lane-operations per unit of work ("VALU roofline"): IEEE basic
# operations (+ - * / sqrt fma min max compare) and integer ops of the numerics contract
# (csrc/rtm.h: Cephes sincos 27, acos/asin 15, atan2 26, normalize 8, quaternion product 19), counted
# on the reference's per-ray arithmetic (Raytracing.cl / MathLib.cl).
VALU_OPS = {
    "box_tests": 25,      # slab test: 6 sub + 6 mul + 10 min/max + entry compare (MathLib.cl:167-199)
    "tri_tests": 56,      # Moller-Trumbore: 2 cross, 4 dot, 1 div, 3 scale, 8 compares (MathLib.cl:117-160)
    "rays": 8,            # 1/d (3 div) + hit bookkeeping
    "ev_diffuse": 141,    # 2 rand, sqrt, sincos, rotateVec + normalize, invPdf, Lambert, origin, attenuation
    "ev_glossy": 239,     # 2 rand, acos, 2 sincos, rotateVec, BRDF_GGX (75), origin, attenuation
    "ev_glass": 28,       # invPdf, origin, attenuation
    "sun_terms": 11,      # Raytracing.cl:115-137 without the IBL lookup
    "env_lookups": 164,   # 2 rotateVec, atan2, asin, texel address + 2x2 mean (MathLib.cl:72-90)
    "samples": 5,         # accumulate + loop
    "pixels": 148,        # genCameraRay (3 rotateVec, normalize), seeds, mean + clamp (Raytracing.cl:18-37, 211-220)
}


def _dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def _profile(config_name: str, ab: str = ""):
    """The newest committed rocprofv3 PMC summary for this workload (profiles/rNN_pmc_<workload>.json;
    ab: an A/B variant's summary, profiles/rNN_ab_<ab>_pmc_<workload>.json)."""
    pat = f"r*_ab_{ab}_pmc_{config_name}.json" if ab else f"r*_pmc_{config_name}.json"
    files = sorted(f for f in glob.glob(os.path.join(ROOT, "profiles", pat)) if ab or "_ab_" not in f)
    if not files:
        return {}
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        d["_file"] = os.path.relpath(files[-1], ROOT)
        return d
    except (OSError, ValueError):
        return {}


def valu_ops(cnt: dict, pixels: int) -> float:
    return float(sum(VALU_OPS[k] * (pixels if k == "pixels" else cnt[k]) for k in VALU_OPS))


def alg_bytes(cnt: dict, wb: dict, pixels: int) -> float:
    # 32 B per box tested (a BVH2 node tests 2, a 4-wide node up to 4, a wide leaf its
    # exact box), 36 B per triangle test, 40 B per ray hit record, 16 B per IBL lookup, + the tile
    # written (12 B per pixel)
    return (cnt["box_tests"] * wb["box_test"] + cnt["tri_tests"] * wb["tri_test"] + cnt["rays"] * wb["ray"]
            + cnt["env_lookups"] * wb["env_lookup"] + pixels * 12.0)


def roofline(ctx, cnt: dict, kernel_ms: float, pixels: int, workload: str, share: float = 1.0) -> dict:
    """share: this launch's fraction of the frame (a rank's tile); the committed PMC summaries are
    whole-frame launches and are scaled by it."""
    info = ctx.scene_info()
    brute = info["brute_records"] > 0
    prof = _profile(workload)
    sec = kernel_ms * 1e-3
    ops = valu_ops(cnt, pixels)
    byt = alg_bytes(cnt, ctx.work_bytes(), pixels)
    traffic = prof.get("hbm_bytes_per_launch")
    issued = prof.get("valu_lane_slots_per_launch")
    traffic = traffic * share if traffic else traffic
    issued = issued * share if issued else issued
    valu = {"achieved": round(ops / sec / 1e12, 3), "peak": VALU_PEAK_TOPS, "unit": "Tops/s",
            "frac": round(ops / sec / 1e12 / VALU_PEAK_TOPS, 4), "alg_ops_per_launch": int(ops),
            "issued": issued, "issued_frac": (round(issued / sec / 1e12 / VALU_PEAK_TOPS, 4) if issued else None)}
    hbm = {"achieved": round(byt / sec / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(byt / sec / 1e9 / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": int(byt),
           "traffic": traffic, "traffic_frac": (round(traffic / sec / 1e9 / HBM_PEAK_GBS, 5) if traffic else None)}
    # tree walk: the algorithmic bytes are served by the vL1D / L2 (C3/C4 L1 hit rate ~90 %), so their
    # rate is priced against the cache hierarchy's delivery ceiling, never against the HBM peak (it would
    # exceed 1); what HBM actually moved is `hbm_measured` (PMC bytes of the same kernel)
    cache = {"achieved": hbm["achieved"], "peak": CACHE_PEAK_GBS, "unit": "GB/s",
             "frac": round(byt / sec / 1e9 / CACHE_PEAK_GBS, 4), "alg_bytes_per_launch": int(byt)}
    main, other, bound = (valu, hbm, "valu") if brute else (cache, valu, "cache")
    out = {"bound": bound}
    out.update(main)
    out["traffic"], out["traffic_frac"] = hbm["traffic"], hbm["traffic_frac"]
    out["hbm_measured"] = {"achieved": (round(traffic / sec / 1e9, 2) if traffic else None), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": hbm["traffic_frac"],
                           "what": "PMC memory-side bytes of the same kernel (reads: 128-byte L2 line fills, "
                                   "calibrated by profiles/r03_hbm_probe.json; + WRITE_SIZE) / kernel time"}
    # the spill-free A/B build of the same walk (4 waves per SIMD, no scratch, 20 LDS stack entries):
    # its memory-side bytes are the walk's own line fills + the frame, i.e. the useful part of the
    # default build's traffic; the rest of the default build's bytes are register spills and stack
    # entries beyond the LDS part
    ab = _profile(workload, "w4")
    if traffic and ab.get("hbm_bytes_per_launch"):
        useful = ab["hbm_bytes_per_launch"] * share
        out["hbm_measured"]["useful"] = {
            "bytes_per_launch": useful, "achieved": round(useful / sec / 1e9, 2), "peak": HBM_PEAK_GBS,
            "frac": round(useful / sec / 1e9 / HBM_PEAK_GBS, 5), "spill_bytes_per_launch": traffic - useful,
            "what": "BVH / triangle line fills + frame writes: the memory-side bytes of the spill-free 4-wave "
                    "build of the same walk (" + ab.get("_file", "") + "), over this build's kernel time"}
    out["kernel_ms"] = round(kernel_ms, 4)
    out["path"] = (f"brute force ({info['brute_boxes']} distinct leaf boxes, {info['brute_records']} triangles)"
                   if brute else f"SAH tree walk ({info['nodes']} nodes, {info['tris']} triangles)")
    if brute:
        # SURVEY 8(d)'s byte model charges HBM for records that this path reads from LDS and the scalar
        # cache: reported as bytes only, never as a fraction of the HBM peak (it would exceed 1)
        out["survey_bytes_model"] = {"alg_bytes_per_launch": hbm["alg_bytes_per_launch"],
                                     "note": "records served from LDS / scalar cache, not HBM: no HBM fraction"}
    else:
        out["other_bound"] = {"bound": "valu", **other}
    out["counts_per_sample"] = {k: round(cnt[k] / max(1, cnt["samples"]), 4)
                                for k in ("box_tests", "tri_tests", "rays", "ev_diffuse", "ev_glossy", "ev_glass",
                                          "sun_terms", "env_lookups", "node_fetches")}
    out["model"] = "VALU_OPS / SURVEY 8(d) bytes per unit in bench.py x counts of the same launch (DESIGN.md 5)"
    if prof:
        out["profile"] = prof.get("_file")
    return out


def host_cores() -> dict:
    """The host CPUs this job may run on: the cgroup CPU quota (cpu.max) when there is one, else the
    affinity mask.  On the GPU box the quota is 16 CPUs of a 256-CPU machine (nproc = 16): more
    threads than that time-slice the same 16 CPUs."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    cores = min(aff, quota) if quota else aff
    return {"cores": cores, "affinity_cpus": aff, "cgroup_cpu_quota": quota, "cpu_count": os.cpu_count()}


def cpu_baseline(wl, scene, ibl, cam, env, target_s: float = 10.0, spp: int = 0, min_s: float = 1.0):
    """Time the CPU oracle on a row sample of the frame (rows 0::step, at the config's spp or at a reduced
    `spp`: the per-sample rate), one OpenMP thread per host CPU the job may use
    (host_cores).  A frame the oracle finishes in under `min_s` (C1) is timed whole, repeated."""
    import oracle.oracle as O
    hc = host_cores()
    threads = hc["cores"]
    spp = int(spp or wl.spp)
    osc = O.OracleScene.from_scene(scene, ibl)
    W = int(cam[6])
    H = (wl.npix + W - 1) // W
    # grow the row sample (rows 0::step) until it takes about target_s, or is the whole frame
    step = 64
    while True:
        t0 = time.perf_counter()
        O.render(osc, cam, env, wl.npix, spp, wl.max_bounce, row0=0, row_step=step, nthreads=threads)
        dt = time.perf_counter() - t0
        if dt >= 0.5 * target_s or step == 1:
            break
        step = max(1, min(step // 2, int(step * dt / target_s)))
    reps = 1
    if step == 1 and dt < 4 * min_s:
        # a frame this short is timed again after that (untimed) first whole-frame pass: the oracle's first
        # pass over a frame runs several times slower than the next ones (0.93 vs 0.18 s for C1 here)
        reps = 0
        t0 = time.perf_counter()
        while reps < 2 or time.perf_counter() - t0 < min_s:
            O.render(osc, cam, env, wl.npix, spp, wl.max_bounce, nthreads=threads)
            reps += 1
        dt = (time.perf_counter() - t0) / reps
    rows = (H + step - 1) // step
    samples = min(rows * W, wl.npix) * spp
    what = "the whole frame" if step == 1 else f"rows 0::{step} of the {W}x{H} frame ({rows} rows)"
    return {"value": round(samples / dt / 1e6, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "host": hc,
            "sample": f"{what} at {spp} spp{'' if spp == wl.spp else f' (config: {wl.spp}; per-sample rate)'}"
                      f" = {samples} samples in {dt:.3f} s{f' (mean of {reps})' if reps > 1 else ''}; "
                      f"oracle/rt_oracle.c (C restatement of the reference kernel), OpenMP",
            "calibration": "C2 in the build container, 8 threads: oracle 1.90 Msamples/s vs the reference kernel "
                           "itself 2.06-2.14 (BASELINE.md 2): 0.89-0.92x (DESIGN.md 5)"}


def gpu_clock() -> dict:
    """The GPU's current / allowed shader clocks from amd-smi (rocm-smi as a fallback), logged beside the
    long timings so that box-to-box clock differences are visible; {} when no tool answers."""
    import re
    import subprocess
    for cmd in (["amd-smi", "metric", "-c"], ["rocm-smi", "--showclocks"]):
        try:
            txt = subprocess.run(cmd, capture_output=True, text=True, timeout=20).stdout
        except (OSError, subprocess.SubprocessError):
            continue
        m = re.search(r"GFX_0:\s*CLK:\s*(\d+)\s*MHz\s*MIN_CLK:\s*(\d+)\s*MHz\s*MAX_CLK:\s*(\d+)", txt, re.S)
        if m:
            return {"tool": cmd[0], "sclk_mhz": int(m.group(1)), "min_mhz": int(m.group(2)), "max_mhz": int(m.group(3))}
        m = re.search(r"sclk.*?(\d+)\s*Mhz", txt, re.I)
        if m:
            return {"tool": cmd[0], "sclk_mhz": int(m.group(1))}
    return {}


class ClockSampler:
    """Polls gpu_clock() on a host thread while a timed region runs (amd-smi is a separate process: the
    GPU's idle clock after a run says nothing, its clock during the frames does)."""

    def __init__(self):
        import threading
        self.samples, self.max_mhz, self._stop = [], None, threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            c = gpu_clock()
            if not c:
                return
            self.samples.append(c["sclk_mhz"])
            self.max_mhz = c.get("max_mhz")
            self._stop.wait(2.0)   # an amd-smi process every 2 s beside the timed frames

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *a):
        self._stop.set()
        self._t.join(timeout=30)

    def summary(self) -> dict:
        if not self.samples:
            return {}
        return {"tool": "amd-smi metric -c (GFX_0), polled during the timed frames", "samples": len(self.samples),
                "sclk_mhz_min": min(self.samples), "sclk_mhz_median": float(np.median(self.samples)),
                "sclk_mhz_max": max(self.samples), "max_mhz": self.max_mhz}


# CPU baseline of each config line: C1 timed in full at its 4 spp, C3-C5 as a per-sample
# rate on a bounded row sample at reduced spp (16: the cached camera ray is ~2 % of a sample's rays)
CPU_SPP = {"C1": 0, "C3": 16, "C4": 16, "C5": 16}


def time_config(ctx_factory, name: str, steps: int, warmup: int, cpu: bool = False):
    """One-GPU device-resident timing of another BASELINE config (C1/C3/C4/C5), same method as the headline;
    every frame is timed on its own (HIP events) and min / median reported beside the mean; with `cpu`,
    the CPU oracle's rate on the same config beside it."""
    import torch
    from ensem3a_openclraytracer_amd import workloads as Wk
    wl = Wk.CONFIGS[name]
    scene, cam, env, npix, spp, mb, ibl = wl.inputs()
    ctx = ctx_factory()
    ctx.set_scene(scene.V_p, scene.V_n, scene.V_uv, scene.faceData, scene.materialData, scene.BVH.exportArray)
    ctx.set_env(ibl)
    out = torch.empty(3 * npix, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for _ in range(warmup):
        ctx.render_device(cam, env, npix, spp, mb, 0, 1, out.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    with ClockSampler() as clk:
        t0 = time.perf_counter()
        for i in range(steps):
            ev[i][0].record(stream)
            ctx.render_device(cam, env, npix, spp, mb, 0, 1, out.data_ptr(), stream.cuda_stream)
            ev[i][1].record(stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
    per = [a.elapsed_time(b) for a, b in ev]
    kernel_ms = float(np.mean(per))
    cnt = ctx.count_work_detail(cam, env, npix, spp, mb)
    rf = roofline(ctx, cnt, kernel_ms, npix, wl.name)
    ctx.close()
    extra = {}
    if cpu:
        cb = cpu_baseline(wl, scene, ibl, cam, env, target_s=6.0, spp=CPU_SPP.get(name, 0))
        extra = {"cpu_baseline": cb, "vs_cpu": round(npix * spp / dt / 1e6 / cb["value"], 1)}
    return {"workload": wl.name, "value": round(npix * spp / dt / 1e6, 3), "unit": "Msamples/s", **extra,
            "ms_per_step": round(dt * 1e3, 3), "steps": steps, "warmup": warmup,
            "frame_ms": {"min": round(min(per), 3), "median": round(float(np.median(per)), 3),
                         "max": round(max(per), 3)},
            "gpu_clock": clk.summary(),
            "roofline": {k: rf.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_frac",
                                                "hbm_measured", "kernel_ms", "path", "profile")},
            "valu_frac": rf["frac"] if rf["bound"] == "valu" else rf["other_bound"]["frac"]}


def cold_call(name: str, device: int) -> dict:
    """SURVEY.md 8(d)'s t_render of a first call: a fresh KernelLauncher (the drop-in path, no torch) and ONE
    launch_Raytracing into a host array, as the Tk UI's first render of a scene runs it (main.py:28,84-86;
    KernelLauncher.py:33-87 pays the uploads on every call): scene validation + SAH / 4-wide packing, the
    uploads, the IBL upload + texel-sum kernel, the render and the read-back.  The process's HIP runtime
    and code objects are already loaded (the benchmark ran before); OBJ parse and the reference BVH
    build are excluded, as in 8(d)."""
    from ensem3a_openclraytracer_amd import workloads as Wk
    from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher
    wl = Wk.CONFIGS[name]
    scene, cam, env, npix, spp, mb, ibl = wl.inputs()
    out = np.zeros(3 * npix, np.float32)
    t0 = time.perf_counter()
    kl = KernelLauncher(None, None, device, None)
    t1 = time.perf_counter()
    kl.launch_Raytracing(out, scene.V_p, scene.V_n, scene.V_uv, scene.faceData, scene.materialData, scene.lightData,
                         scene.BVH.exportArray, cam, env, npix, spp, mb, ibl)
    t2 = time.perf_counter()
    tm = kl.native.timings()
    kl.close()
    call_ms = (t2 - t1) * 1e3
    parts = {k: round(v, 3) for k, v in tm.items()}
    parts["create_ms"] = round((t1 - t0) * 1e3, 3)
    parts["other_ms"] = round(call_ms - sum(tm.values()), 3)   # argument checks + the upload cache's hashes
    return {"value": round(npix * spp / (call_ms * 1e-3) / 1e6, 3), "unit": "Msamples/s", "ms": round(call_ms, 3),
            "split": parts, "what": "fresh KernelLauncher + one launch_Raytracing into host memory: pack + uploads + "
                                    "IBL + render + read-back (create_ms, the rt_create, is outside 'ms')"}


def two_frames_in_flight(ctx, make_ctx, scene, ibl, cam, env, npix, spp, mb, steps, warmup) -> dict:
    """Frames of a sequence (an animation, or a UI re-rendering) rendered on two contexts and two
    streams alternately, so that one frame's kernel fills the CUs its predecessor's tail leaves idle
    (frame tail).  Reported beside the headline, never as `value`: the headline renders
    one frame at a time, as launch_Raytracing does."""
    import torch
    ctx2 = make_ctx()
    try:
        ctx2.set_scene(scene.V_p, scene.V_n, scene.V_uv, scene.faceData, scene.materialData, scene.BVH.exportArray)
        ctx2.set_env(ibl)
        lanes = [(ctx, torch.cuda.Stream()), (ctx2, torch.cuda.Stream())]
        outs = [torch.empty(3 * npix, dtype=torch.float32, device="cuda") for _ in lanes]

        def run(n):
            for f in range(n):
                c, s = lanes[f % 2]
                c.render_device(cam, env, npix, spp, mb, 0, 1, outs[f % 2].data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()

        run(max(warmup, 2))
        t0 = time.perf_counter()
        run(steps)
        dt = (time.perf_counter() - t0) / steps
    finally:
        ctx2.close()
    return {"value": round(npix * spp / dt / 1e6, 3), "unit": "Msamples/s", "ms_per_frame": round(dt * 1e3, 4),
            "steps": steps, "what": "consecutive frames alternating over two contexts / streams (frame k+1 starts "
                                    "while frame k drains); not the headline, which renders one frame at a time"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--traversal", default="fast", choices=["fast", "ref"])
    ap.add_argument("--bvh", default="sah", choices=["sah", "reference"])
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--option", action="append", default=[], help="rt_set_option KEY=VALUE (repeatable)")
    ap.add_argument("--bvh-width", type=int, default=0, choices=[0, 2, 4],
                    help="FAST tree walk layout: 2 = BVH2, 4 = 4-wide quantised (0 = library default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C3/C4 lines and the host-boundary timing")
    ap.add_argument("--no-counts", action="store_true",
                    help="skip the instrumented work-count launch (and the roofline it feeds): profiling passes")
    ap.add_argument("--check", action="store_true",
                    help="N>1: rank 0 re-renders the whole frame alone and compares it with the gathered one")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from ensem3a_openclraytracer_amd import _native
    from ensem3a_openclraytracer_amd import distributed as D
    from ensem3a_openclraytracer_amd import workloads as Wk

    rank, world, local = _dist_env()
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    world = max(world, 1)
    # Rehearsal of the N>1 path on a one-GPU box: every rank on device 0 and the collectives over gloo
    # on host copies (RCCL refuses two ranks on one GPU).  Never used for measured runs.
    rehearsal = os.environ.get("BENCH_SAME_DEVICE") == "1"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    coll = "cpu" if rehearsal else "cuda"   # where collective buffers live

    def make_ctx():
        c = _native.Context(device_ids=[local])
        c.set_option("traversal", _native.RT_TRAVERSAL_FAST if args.traversal == "fast" else _native.RT_TRAVERSAL_REF)
        c.set_option("bvh", _native.RT_BVH_SAH if args.bvh == "sah" else _native.RT_BVH_REFERENCE)
        if args.block:
            c.set_option("block", args.block)
        if args.bvh_width:
            c.set_option("bvh_width", args.bvh_width)
        for kv in args.option:
            k, v = kv.split("=")
            c.set_option(k, int(v))
        return c

    def run_frames(ctx, cam, env, npix, spp, mb, steps, warmup):
        """Render `steps` frames of one config after `warmup` untimed ones: every rank its row tile
        (rt_render_device, scene resident), rank 0 gathers the tiles over RCCL and assembles each frame
        (frame k's gather overlaps frame k+1's render: two tile buffers).  Returns (elapsed s, mean
        kernel ms, the last assembled frame on rank 0), both times the max over ranks."""
        width = int(cam[6])
        stream = torch.cuda.current_stream()
        mrows = D.max_tile_rows(npix, width, world)
        nbuf = 2 if world > 1 else 1
        tiles = [torch.zeros(3 * width * mrows, dtype=torch.float32, device="cuda") for _ in range(nbuf)]
        bufs = [[torch.empty(tiles[0].numel(), dtype=torch.float32, device=coll) for _ in range(world)]
                for _ in range(nbuf)] if (world > 1 and rank == 0) else [None] * nbuf
        frame = torch.empty(3 * npix, dtype=torch.float32, device=coll) if (rank == 0 and world > 1) else None
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        pending = []   # (work, buffer index) of the gather in flight

        def finish_pending():
            while pending:
                work, b = pending.pop(0)
                if work is not None:
                    work.wait()   # the current stream waits for the gather (no host block for RCCL)
                if rank == 0:
                    D.assemble(bufs[b], width, npix, world, out=frame)

        def step(i=None, k=0):
            b = k % nbuf
            if i is not None:
                ev[i][0].record(stream)
            ctx.render_device(cam, env, npix, spp, mb, rank, world, tiles[b].data_ptr(), stream.cuda_stream)
            if i is not None:
                ev[i][1].record(stream)
            if world > 1:
                if coll == "cuda":
                    work = dist.gather(tiles[b], gather_list=bufs[b], dst=0, async_op=True)
                else:   # one-GPU gloo rehearsal: host copies, synchronous
                    dist.gather(tiles[b].cpu(), gather_list=bufs[b], dst=0)
                    work = None
                finish_pending()      # the previous frame's gather ran while this frame rendered
                pending.append((work, b))

        for w in range(warmup):
            step(k=w)
        finish_pending()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i, k=i)
        finish_pending()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        kms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        if world > 1:
            tt = torch.tensor([elapsed, kms], dtype=torch.float64, device=coll)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed, kms = float(tt[0]), float(tt[1])
        return elapsed, kms, frame

    wl = Wk.CONFIGS[args.config]
    scene, cam, env, npix, spp, mb, ibl = wl.inputs()
    ctx = make_ctx()
    ctx.set_scene(scene.V_p, scene.V_n, scene.V_uv, scene.faceData, scene.materialData, scene.BVH.exportArray)
    ctx.set_env(ibl)
    width = int(cam[6])
    stream = torch.cuda.current_stream()
    elapsed, kernel_ms, frame = run_frames(ctx, cam, env, npix, spp, mb, args.steps, args.warmup)

    # work counters of the same traversal on this rank's tile (instrumented launch, not timed)
    tile_pixels = D.tile_rows(npix, width, rank, world) * width
    rf = None
    if not args.no_counts:
        cnt = ctx.count_work_detail(cam, env, npix, spp, mb, rank, world)
        rf = roofline(ctx, cnt, kernel_ms, tile_pixels, wl.name, share=tile_pixels / npix)

    frame_check = None
    if args.check and world > 1:
        _, _, frame = run_frames(ctx, cam, env, npix, spp, mb, 1, 0)
        if rank == 0:
            full = torch.empty(3 * npix, dtype=torch.float32, device="cuda")
            ctx.render_device(cam, env, npix, spp, mb, 0, 1, full.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            frame_check = "bit-identical" if torch.equal(full.to(coll), frame) else "MISMATCH"
        dist.barrier()

    # N > 1: the other BASELINE configs through the same multi-GPU path (row tiles + RCCL gather), so the
    # driver's per-N runs measure every config's strong scaling, not only the headline's
    multi_cfg = {}
    if world > 1 and not args.no_extra and args.config == "C2":
        for c, st, wu in (("C3", 2, 1), ("C4", 2, 1), ("C5", 1, 1)):
            wlc = Wk.CONFIGS[c]
            sc_c, cam_c, env_c, npix_c, spp_c, mb_c, ibl_c = wlc.inputs()
            cc = make_ctx()
            cc.set_scene(sc_c.V_p, sc_c.V_n, sc_c.V_uv, sc_c.faceData, sc_c.materialData, sc_c.BVH.exportArray)
            cc.set_env(ibl_c)
            el, kms, _ = run_frames(cc, cam_c, env_c, npix_c, spp_c, mb_c, st, wu)
            cc.close()
            multi_cfg[c] = {"workload": wlc.name, "value": round(npix_c * spp_c * st / el / 1e6, 3),
                            "unit": "Msamples/s", "ms_per_step": round(el / st * 1e3, 3), "steps": st, "warmup": wu,
                            "kernel_ms_max_rank": round(kms, 3),
                            "parallelism": f"row-interleaved x{world}" + (" + gloo gather (one-GPU rehearsal)"
                                                                          if rehearsal else " + RCCL gather")}

    if rank == 0:
        samples = npix * spp
        ms_per_step = elapsed / args.steps * 1e3
        value = samples * args.steps / elapsed / 1e6
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": wl.data_note(),
            "config": {"workload": wl.name, "scene": wl.scene, "width": wl.width, "height": wl.height,
                       "spp": spp, "max_bounce": mb, "traversal": args.traversal, "bvh": args.bvh,
                       "parallelism": f"row-interleaved x{world}" + (
                           (" + gloo gather (one-GPU rehearsal)" if rehearsal else " + RCCL gather") if world > 1 else "")},
            "roofline": rf,
        }
        if frame_check is not None:
            line["frame_check"] = f"gathered {world}-rank frame vs one-device render: {frame_check}"
        if multi_cfg:
            line["configs"] = multi_cfg
        if world == 1 and not args.no_extra:
            # the drop-in boundary's own rate: blocking rt_render into host memory (kernel + read-back),
            # same warmup / steps as the headline
            host = np.zeros(3 * npix, np.float32)
            for _ in range(args.warmup):
                ctx.render(cam, env, npix, spp, mb, out=host)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                ctx.render(cam, env, npix, spp, mb, out=host)
            dt = (time.perf_counter() - t0) / args.steps
            line["host_boundary"] = {"value": round(samples / dt / 1e6, 3), "unit": "Msamples/s",
                                     "ms_per_frame": round(dt * 1e3, 3), "steps": args.steps,
                                     "what": "rt_render (launch_Raytracing's C-ABI): kernel + copy of the frame "
                                             "into caller memory, scene already uploaded"}
        if world == 1 and not args.no_extra:
            line["two_frames_in_flight"] = two_frames_in_flight(ctx, make_ctx, scene, ibl, cam, env, npix, spp, mb,
                                                                args.steps, args.warmup)
        if world == 1 and not args.no_extra and args.config == "C2":
            ctx.close()
            ctx = None
            cpu = not args.no_cpu_baseline
            line["configs"] = {"C1": time_config(make_ctx, "C1", 20, 3, cpu)}
            # C3 / C4 over 5 frames (about 0.5 / 1.4 s: their frames spread 1-3 % within a run), C5 over 2
            line["configs"].update({c: time_config(make_ctx, c, st, 1, cpu) for c, st in (("C3", 5), ("C4", 5), ("C5", 2))})
            line["configs"]["C2"] = {"workload": wl.name, "value": line["value"], "unit": "Msamples/s",
                                     "note": "the headline above"}
            for c in ("C1", "C2", "C3", "C4", "C5"):
                line["configs"][c]["cold_call"] = cold_call(c, local)
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(wl, scene, ibl, cam, env)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if ctx is not None:
        ctx.close()


if __name__ == "__main__":
    main()
