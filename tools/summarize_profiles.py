"""Summarise rocprofv3 passes of bench.py into profiles/ (committed evidence).

    python tools/summarize_profiles.py gpurun_out/SESSION:CFG[:OPTS] TAG WORKLOAD [FRAMES]
        the kt / pmc steps of tools/gpu_session.py (gpurun_out/SESSION_kt_CFG[_OPTS],
        SESSION_pmc_CFG_GROUP[_OPTS]; OPTS = the step's option suffix, e.g. slices-8)
    python tools/summarize_profiles.py DIR TAG WORKLOAD [FRAMES]
        DIR/kt, DIR/fetch, DIR/write, DIR/req, DIR/sq, DIR/hit (one pass each)
    --wave-stats FILE:CONFIG  also record the SIMD efficiency of the render loop (tools/wave_stats.py's
        JSON line for CONFIG in FILE: trav_simd_eff = items advanced per lane-step of the traversal, beside
        valu_lane_util, which the predicated steps inflate)
FRAMES (bench warmup + steps) is required when several render-kernel instantiations ran (two-pass
launches), since a frame is then several dispatches.

Writes profiles/TAG_kernel_stats_WORKLOAD.csv (the --stats table of the kernel-trace run) and
profiles/TAG_pmc_WORKLOAD.json: per-launch means of every counter of the render kernel, and
  hbm_read_bytes_per_launch = 128 x TCC_EA0_RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B: the bytes the
      L2 moved from memory (HBM or the Infinity Cache), every request at its size.  Calibrated by
      tools/hbm_probe.hip (profiles/r03_hbm_probe.json): on gfx950 the L2 fetches a whole 128-byte line
      per miss, for 16-byte streaming reads and for 16/64/128-byte random gathers alike, and the
      by-size sum equals the known bytes of a 128-byte gather and of a streaming read (0.999-1.000);
      FETCH_SIZE tallies each 128-byte request at 64 B (TCC_BUBBLE reads 0), i.e. exactly half.  A
      64-byte record gathered at random therefore costs 128 bytes of memory traffic, two records'
      worth (hbm_line_bytes_per_request = 128).  Without the request-size pass: 2 x FETCH_SIZE.
  hbm_bytes_per_launch = hbm_read_bytes_per_launch + WRITE_SIZE (writes: exact for streaming
      stores, MI355X_MICROARCH.md);
  valu_lane_slots_per_launch = SQ_INSTS_VALU x 64 (wave-level VALU instructions x lanes);
  valu_lane_util = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU) (active lanes per VALU issue);
  valu_issue_frac = valu_lane_slots_per_launch / kernel time / 78.64e12 lane-ops/s.
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# FAST, uninstrumented (any variant): the megakernels
KERNEL = r"render(_resume)?_kernel<(0, )?false, false|wave_kernel<false"
GROUPS = ("fetch", "write", "dram", "req", "sq", "hit")


def _rows(pattern):
    out = []
    for p in glob.glob(pattern):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def main(prof, tag, workload, frames=None, kernel=KERNEL, wave_stats=None):
    """frames: frames the profiled run rendered (bench warmup + steps).  A frame may take several
    dispatches of the render kernel (two-pass launches, option "pilot"); every *_per_launch value and
    kernel_avg_ms are then per frame (totals / frames).  Default: one dispatch per frame."""
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    if ":" in prof:   # tools/gpu_session.py layout
        pre, cfg, *opt = prof.split(":")
        sfx = "_" + opt[0] if opt and opt[0] else ""
        where = {"kt": f"{pre}_kt_{cfg}{sfx}", **{g: f"{pre}_pmc_{cfg}_{g}{sfx}" for g in GROUPS}}
    else:
        where = {g: os.path.join(prof, g) for g in ("kt",) + GROUPS}
    stats = glob.glob(os.path.join(where["kt"], "*kernel_stats.csv"))
    if not stats:   # a run that never produced its kernel trace must not overwrite committed summaries
        sys.exit(f"no kernel trace under {where['kt']}")
    s = {"workload": workload, "kernel": kernel, "source": "rocprofv3 (tools/gpu_session.py kt / pmc steps)"}
    if stats:
        # every instantiation of the render kernel counts (two-pass launches: pass 1 and pass 2; a
        # device-chosen team size launches the other sizes' instantiations, which return at once)
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats_{workload}.csv"))
        names, calls, total = [], 0, 0.0
        for r in _rows(stats[0]):
            if re.search(kernel, r["Name"]):
                names.append(r["Name"][:120])
                calls += int(r["Calls"])
                total += float(r["TotalDurationNs"])
        if len(names) > 1 and not frames:
            sys.exit(f"{len(names)} render-kernel instantiations matched: give FRAMES (frames the run rendered)")
        if names:
            s["kernel_name"] = names[0] if len(names) == 1 else names
            s["kernel_calls"] = calls
            s["frames"] = int(frames) if frames else calls
            s["kernel_avg_ms"] = total / 1e6 / s["frames"]
    counters, dispatches = {}, {}
    for sub in GROUPS:
        for r in _rows(os.path.join(where[sub], "*counter_collection.csv")):
            if re.search(kernel, r["Kernel_Name"]):
                counters.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
                dispatches.setdefault(r["Counter_Name"], set()).add(r["Dispatch_Id"])
    # dispatches per frame from the kernel trace; a pass may render a different number of frames than
    # the kernel-trace run (e.g. 20 timed steps traced, 1 per counter pass), so each counter is divided
    # by the frames of its own pass
    per_frame = s.get("kernel_calls", 1) / max(1, s.get("frames", 1))
    for k, v in sorted(counters.items()):
        # per frame: every dispatch of the frame summed
        nfr = max(1.0, len(dispatches[k]) / per_frame)
        s[k + "_per_launch"] = float(np.sum(v)) / nfr
        s[k + "_launches"] = len(v)
    g = lambda k: s.get(k + "_per_launch")  # noqa: E731
    if g("TCC_EA0_RDREQ_128B_sum") is not None:
        s["hbm_read_bytes_per_launch"] = (128.0 * g("TCC_EA0_RDREQ_128B_sum") + 64.0 * (g("TCC_EA0_RDREQ_64B_sum") or 0.0)
                                          + 32.0 * (g("TCC_EA0_RDREQ_32B_sum") or 0.0))
        s["hbm_read_note"] = "128 x RDREQ_128B + 64 x RDREQ_64B + 32 x RDREQ_32B (profiles/r03_hbm_probe.json)"
    elif g("FETCH_SIZE") is not None:
        s["hbm_read_bytes_per_launch"] = 2.0 * g("FETCH_SIZE") * 1024
        s["hbm_read_note"] = "2 x FETCH_SIZE KiB (every request a 128-byte line, profiles/r03_hbm_probe.json)"
    if s.get("hbm_read_bytes_per_launch") is not None and g("WRITE_SIZE") is not None:
        s["hbm_bytes_per_launch"] = s["hbm_read_bytes_per_launch"] + g("WRITE_SIZE") * 1024
        s["hbm_bytes_note"] = "memory-side reads (128-byte lines, calibrated) + WRITE_SIZE"
        if s.get("kernel_avg_ms"):
            s["hbm_GBps"] = s["hbm_bytes_per_launch"] / (s["kernel_avg_ms"] * 1e-3) / 1e9
            s["hbm_frac_of_8TBps"] = s["hbm_GBps"] / 8000.0
    if g("SQ_INSTS_VALU") is not None:
        s["valu_lane_slots_per_launch"] = 64.0 * g("SQ_INSTS_VALU")
        if g("SQ_ACTIVE_INST_VALU"):
            s["valu_lane_util"] = g("SQ_THREAD_CYCLES_VALU") / (64.0 * g("SQ_ACTIVE_INST_VALU"))
        if s.get("kernel_avg_ms"):
            s["valu_issue_frac"] = s["valu_lane_slots_per_launch"] / (s["kernel_avg_ms"] * 1e-3) / 78.6432e12
    if wave_stats:
        path, cfg = wave_stats.rsplit(":", 1)
        with open(path) as f:
            rows = [json.loads(ln) for ln in f if ln.strip()]
        row = [r for r in rows if r["config"] == cfg and not r.get("opts")][-1]
        for k in ("trav_simd_eff", "trav_iters_per_wave_render_iter", "rays_per_lane_render_iter", "trav_cycle_share"):
            s[k] = row[k]
        s["wave_stats_note"] = "tools/wave_stats.py (instrumented kernel, product defaults): " + os.path.basename(path)
    if g("TCC_REQ_sum"):
        s["l2_hit_rate"] = g("TCC_HIT_sum") / max(1.0, g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc_{workload}.json"), "w") as f:
        json.dump(s, f, indent=1)
    print(json.dumps(s, indent=1))


if __name__ == "__main__":
    args = sys.argv[1:]
    ws = None
    if "--wave-stats" in args:
        i = args.index("--wave-stats")
        ws = args[i + 1]
        del args[i:i + 2]
    main(*args[:4], wave_stats=ws)
