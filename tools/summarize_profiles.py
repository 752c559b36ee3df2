"""Summarise rocprofv3 output of tools/run_profiles.sh into profiles/ (committed evidence).

    python tools/summarize_profiles.py gpurun_out/prof TAG WORKLOAD

Writes profiles/TAG_kernel_stats_WORKLOAD.csv (the --stats table of the kernel-trace run)
and profiles/TAG_pmc_WORKLOAD.json: per-launch counters of the render kernel and the HBM
bytes per launch, corrected as MI355X_MICROARCH.md prescribes for gfx950 (FETCH_SIZE is in
KiB and reads 1/2 of a wide streaming read's bytes -> x2; WRITE_SIZE in KiB, exact).
"""
import csv
import re
import glob
import json
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = r"render(_resume)?_kernel<(0, )?false, false"  # FAST, uninstrumented (any variant)


def _rows(pattern):
    out = []
    for p in glob.glob(pattern):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def main(prof, tag, workload, kernel=KERNEL):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = glob.glob(os.path.join(prof, "kt", "*kernel_stats.csv"))
    summary = {"workload": workload, "kernel": kernel, "source": "rocprofv3 (tools/run_profiles.sh)"}
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, "profiles", f"{tag}_kernel_stats_{workload}.csv"))
        for r in _rows(stats[0]):
            if re.search(kernel, r["Name"]):
                summary["kernel_calls"] = int(r["Calls"])
                summary["kernel_avg_ms"] = float(r["AverageNs"]) / 1e6
    counters = {}
    for sub in ("fetch", "write", "dram"):
        for r in _rows(os.path.join(prof, sub, "*counter_collection.csv")):
            if re.search(kernel, r["Kernel_Name"]):
                counters.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in counters.items():
        summary[k + "_per_launch"] = float(np.mean(v))
        summary[k + "_launches"] = len(v)
    if "FETCH_SIZE_per_launch" in summary and "WRITE_SIZE_per_launch" in summary:
        summary["hbm_bytes_per_launch"] = (2.0 * summary["FETCH_SIZE_per_launch"] + summary["WRITE_SIZE_per_launch"]) * 1024
        summary["hbm_bytes_note"] = ("FETCH_SIZE x2 (gfx950 half-count correction for wide reads; this kernel's "
                                     "narrow gathers are uncalibrated) + WRITE_SIZE, KiB -> bytes")
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc_{workload}.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
