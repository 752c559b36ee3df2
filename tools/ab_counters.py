"""Counters of an A/B pair of builds or option sets, from tools/gpu_session.py pmc steps (committed evidence).

    python tools/ab_counters.py OUT.json "WHAT" NAME=SESSION[:OPTS] NAME=SESSION[:OPTS] ... -- CFG[=FRAMES] ...

For every NAME (a session tag whose pmc steps ran the build / options of that variant) and every CFG,
the counters of the render dispatches (render_resume_kernel, render_kernel, spec_kernel: every
dispatch of a frame) of gpurun_out/SESSION_pmc_CFG_GROUP[_OPTS]/ are summed and divided by FRAMES
(bench warmup + steps: 2 by default), and the derived rates written:
  kernel_ms              render-dispatch time per frame (from the dispatch timestamps of the sq pass)
  valu_issue_frac        SQ_INSTS_VALU x 64 / (kernel time x 78.64e12 lane-slots/s)
  valu_lane_util         SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU): lanes active per VALU issue
  wait_frac              SQ_WAIT_ANY / SQ_WAVE_CYCLES: wave-cycles waiting on a counter
  ta_busy_frac           TA_TA_BUSY_sum / (32 x GRBM_GUI_ACTIVE) (the normalisation of the r03 summaries)
  vmem_rd_per_frame      SQ_INSTS_VMEM_RD (wave-level vector-memory read instructions)
  stall                  (the stall pass) wave-cycles issuing / parked on a counter / ready but not issued
                         (SQ_ACTIVE_INST_ANY, SQ_WAIT_ANY, SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES: disjoint)
"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = re.compile(r"render(_resume)?_kernel<(0, )?false, false|spec_kernel<")
PEAK = 78.6432e12


def sums(path):
    tot, t = {}, 0.0
    seen = set()
    for f in glob.glob(os.path.join(path, "*counter_collection.csv")):
        for r in csv.DictReader(open(f, newline="")):
            if not KERNEL.search(r["Kernel_Name"]):
                continue
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if r["Dispatch_Id"] not in seen:
                seen.add(r["Dispatch_Id"])
                t += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return tot, t, len(seen)


def main():
    out, what = sys.argv[1], sys.argv[2]
    k = sys.argv.index("--")
    variants = [a.split("=", 1) for a in sys.argv[3:k]]
    cfgs = [c.split("=") for c in sys.argv[k + 1:]]
    res = {"what": what, "rows": {}}
    for name, spec in variants:
        sess, _, opts = spec.partition(":")
        for cfg in cfgs:
            c, frames = cfg[0], int(cfg[1]) if len(cfg) > 1 else 2
            suf = ("_" + opts) if opts else ""
            row = {}
            sq, t, nd = sums(os.path.join(ROOT, "gpurun_out", f"{sess}_pmc_{c}_sq{suf}"))
            ta, _, _ = sums(os.path.join(ROOT, "gpurun_out", f"{sess}_pmc_{c}_ta{suf}"))
            stall, t2, nd2 = sums(os.path.join(ROOT, "gpurun_out", f"{sess}_pmc_{c}_stall{suf}"))
            if stall:
                wc = stall["SQ_WAVE_CYCLES"]
                row["stall"] = {
                    "kernel_ms": round(t2 / frames * 1e3, 3),
                    "active_frac": round(stall["SQ_ACTIVE_INST_ANY"] / wc, 4),     # wave-cycles issuing
                    "wait_frac": round(stall["SQ_WAIT_ANY"] / wc, 4),              # parked in s_waitcnt / barrier
                    "wait_inst_frac": round(stall["SQ_WAIT_INST_ANY"] / wc, 4),    # ready but not issued (pipe / dependency)
                    "wait_inst_lds_frac": round(stall["SQ_WAIT_INST_LDS"] / wc, 4),
                    "valu_issue_frac": round(stall["SQ_INSTS_VALU"] * 64 / t2 / PEAK, 4),
                    "per_frame": {k: stall[k] / frames for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS")},
                }
            if ta:
                row["ta_busy_frac"] = round(ta["TA_TA_BUSY_sum"] / (32 * ta["GRBM_GUI_ACTIVE"]), 4)
                row["vmem_rd_per_frame"] = ta["SQ_INSTS_VMEM_RD"] / frames
                row["valu_per_frame"] = ta["SQ_INSTS_VALU"] / frames
                _, tt, _ = sums(os.path.join(ROOT, "gpurun_out", f"{sess}_pmc_{c}_ta{suf}"))
                row["ta_pass_kernel_ms"] = round(tt / frames * 1e3, 3)
            if not sq:
                if stall or ta:
                    res["rows"][f"{name} {c}"] = row
                continue
            row["dispatches"] = nd
            row["kernel_ms"] = round(t / frames * 1e3, 3)
            row["valu_issue_frac"] = round(sq["SQ_INSTS_VALU"] * 64 / t / PEAK, 4)
            row["valu_lane_util"] = round(sq["SQ_THREAD_CYCLES_VALU"] / (64 * sq["SQ_ACTIVE_INST_VALU"]), 4)
            row["wait_frac"] = round(sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"], 4)
            row["SQ_INSTS_VALU_per_frame"] = sq["SQ_INSTS_VALU"] / frames
            res["rows"][f"{name} {c}"] = row
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
