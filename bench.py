"""Benchmark of the path-tracing hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--traversal fast|ref] [--bvh sah|reference]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one full frame of the configuration (default C2: Cornell box
1024x1024, 64 spp, maxBounce 4): every rank renders its row-interleaved tile with
the HIP kernel (scene and IBL already resident in HBM), rank 0 gathers the tiles
over RCCL and assembles the frame.  K steps are timed between barrier +
synchronize fences; the max over ranks is reported.  value = W*H*spp / time in
Msamples/s (whole job; the frame size is fixed, so scaling is "strong").

Extra fields:
  roofline     -- dominant kernel (render_kernel): algorithmic bytes per launch
                  (this build's own traversal counters x bytes per unit, see
                  DESIGN.md) / average kernel time from HIP events on the launch
                  stream; peak = 8 TB/s HBM; traffic = PMC-measured HBM bytes per
                  launch from profiles/ (rocprofv3) when present, else null;
                  traffic_frac = that measured traffic / kernel time / peak.  On a
                  cache-resident scene (C2) frac > 1: the algorithmic bytes are
                  served from LDS / scalar cache / L2, not HBM.
  cpu_baseline -- the CPU oracle (a C restatement of the reference kernel, OpenMP)
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
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def _dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def _pmc_traffic(config_name: str):
    """Per-launch HBM bytes from the newest committed rocprofv3 PMC summary for this workload."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc*{config_name}*.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(wl, scene, ibl, cam, env, target_s: float = 10.0):
    """Time the CPU oracle on a row sample of the frame (rows row0::step at full spp)."""
    import oracle.oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    osc = O.OracleScene.from_scene(scene, ibl)
    W = int(cam[6])
    H = (wl.npix + W - 1) // W
    # grow the row sample (rows 0::step) until it takes about target_s, or is the whole frame
    step = 64
    while True:
        t0 = time.perf_counter()
        O.render(osc, cam, env, wl.npix, wl.spp, wl.max_bounce, row0=0, row_step=step, nthreads=threads)
        dt = time.perf_counter() - t0
        if dt >= 0.5 * target_s or step == 1:
            break
        step = max(1, min(step // 2, int(step * dt / target_s)))
    rows = (H + step - 1) // step
    samples = rows * W * wl.spp
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"rows 0::{step} of the {W}x{H} frame ({rows} rows) at {wl.spp} spp = {samples} samples "
                      f"in {dt:.2f} s; oracle/rt_oracle.c (C restatement of the reference kernel), OpenMP"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--traversal", default="fast", choices=["fast", "ref"])
    ap.add_argument("--bvh", default="sah", choices=["sah", "reference"])
    ap.add_argument("--block", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
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

    wl = Wk.CONFIGS[args.config]
    scene, cam, env, npix, spp, mb, ibl = wl.inputs()
    ctx = _native.Context(device_ids=[local])
    ctx.set_option("traversal", _native.RT_TRAVERSAL_FAST if args.traversal == "fast" else _native.RT_TRAVERSAL_REF)
    ctx.set_option("bvh", _native.RT_BVH_SAH if args.bvh == "sah" else _native.RT_BVH_REFERENCE)
    if args.block:
        ctx.set_option("block", args.block)
    ctx.set_scene(scene.V_p, scene.V_n, scene.V_uv, scene.faceData, scene.materialData, scene.BVH.exportArray)
    ctx.set_env(ibl)
    width = int(cam[6])
    stream = torch.cuda.current_stream()
    mrows = D.max_tile_rows(npix, width, world)
    tile = torch.zeros(3 * width * mrows, dtype=torch.float32, device="cuda")
    bufs = [torch.empty(tile.numel(), dtype=torch.float32, device=coll) for _ in range(world)] \
        if (world > 1 and rank == 0) else None
    frame = torch.empty(3 * npix, dtype=torch.float32, device=coll) if (rank == 0 and world > 1) else None
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev[i][0].record(stream)
        ctx.render_device(cam, env, npix, spp, mb, rank, world, tile.data_ptr(), stream.cuda_stream)
        if i is not None:
            ev[i][1].record(stream)
        if world > 1:
            dist.gather(tile if coll == "cuda" else tile.cpu(), gather_list=bufs, dst=0)
            if rank == 0:
                D.assemble(bufs, width, npix, world, out=frame)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        tt = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=coll)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(tt[0]), float(tt[1])

    # algorithmic bytes of one launch on this rank: counters of the same traversal x bytes per unit
    # The bytes are those of the tree walk (FAST over the SAH BVH2): scenes of <= 64 triangles run the
    # lock-step brute-force path instead, which reads every triangle record per ray from the scalar
    # cache -- more bytes by construction, so it is not what the roofline is priced on.
    ctx.set_option("brute_max", 0)
    cnt = ctx.count_work(cam, env, npix, spp, mb, rank, world)
    ctx.set_option("brute_max", 64)
    wb = ctx.work_bytes()
    alg_bytes = (cnt["node_fetches"] * wb["node_fetch"] + cnt["tri_tests"] * wb["tri_test"]
                 + cnt["rays"] * wb["ray"] + cnt["env_lookups"] * wb["env_lookup"]
                 + D.tile_rows(npix, width, rank, world) * width * 12)   # + the tile written
    if world > 1:
        tb = torch.tensor([alg_bytes], dtype=torch.float64, device=coll)
        dist.all_reduce(tb, op=dist.ReduceOp.MAX)
        alg_bytes = float(tb[0])

    frame_check = None
    if args.check and world > 1:
        step()
        torch.cuda.synchronize()
        if rank == 0:
            full = torch.empty(3 * npix, dtype=torch.float32, device="cuda")
            ctx.render_device(cam, env, npix, spp, mb, 0, 1, full.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            frame_check = "bit-identical" if torch.equal(full.to(coll), frame) else "MISMATCH"
        dist.barrier()

    if rank == 0:
        samples = npix * spp
        ms_per_step = elapsed / args.steps * 1e3
        value = samples * args.steps / elapsed / 1e6
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
        traffic = _pmc_traffic(wl.name)   # measured HBM bytes per launch (committed rocprofv3 PMC summary)
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": wl.data_note(),
            "config": {"workload": wl.name, "scene": wl.scene, "width": wl.width, "height": wl.height,
                       "spp": spp, "max_bounce": mb, "traversal": args.traversal, "bvh": args.bvh,
                       "parallelism": f"row-interleaved x{world}" + (
                           (" + gloo gather (one-GPU rehearsal)" if rehearsal else " + RCCL gather") if world > 1 else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_frac": (round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                                          if traffic else None),
                         "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": int(alg_bytes),
                         "bytes_model": "SURVEY 8(d): 32 B/box tested (FAST node = 2 boxes), 36 B/triangle test, "
                                        "40 B/ray hit record, 16 B/IBL lookup; counts of this build's SAH tree walk",
                         "counts_per_sample": {k: round(v / (samples / world), 4) for k, v in cnt.items()}},
        }
        if frame_check is not None:
            line["frame_check"] = f"gathered {world}-rank frame vs one-device render: {frame_check}"
        if world == 1:
            # the drop-in boundary's own rate: blocking rt_render into host memory (kernel + PCIe read-back)
            host = np.zeros(3 * npix, np.float32)
            ctx.render(cam, env, npix, spp, mb, out=host)
            t0 = time.perf_counter()
            for _ in range(3):
                ctx.render(cam, env, npix, spp, mb, out=host)
            dt = (time.perf_counter() - t0) / 3
            line["host_boundary"] = {"value": round(samples / dt / 1e6, 3), "unit": "Msamples/s",
                                     "ms_per_frame": round(dt * 1e3, 3),
                                     "what": "rt_render (launch_Raytracing's C-ABI): kernel + device-to-host copy "
                                             "of the frame into caller memory, scene already uploaded"}
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(wl, scene, ibl, cam, env)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
