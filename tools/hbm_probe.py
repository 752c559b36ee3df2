"""Calibration of the L2 memory-side byte counters on reads of known size (tools/hbm_probe.hip).

    python tools/hbm_probe.py run OUTDIR -- PROGRAM [ARGS...]   (GPU box: one rocprofv3 pass per counter group)
    python tools/hbm_probe.py summary OUTDIR [OUT_JSON]         (-> profiles/r03_hbm_probe.json)

For every probe kernel (its second dispatch: the first warms the TLB): the known bytes it reads, each
counter, and the byte figures they imply --
  fetch_size_bytes      FETCH_SIZE x 1024 (rocprofv3's derived counter, as reported)
  rdreq_x64             TCC_EA0_RDREQ x 64 B
  rdreq_by_size         32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (requests tallied at their size)
  dram_32b_x32          TCC_EA0_RDREQ_DRAM_32B x 32 B (32-byte units of the DRAM-bound reads)
and the ratio of each to the known bytes, so that the correction applied to the render kernels'
counters (tools/summarize_profiles.py) rests on a measured calibration of the same access shape.
"""
import csv
import re
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# one counter group per rocprofv3 run (at most 4 TCC counters a pass)
PASSES = {
    "kt": ["--kernel-trace", "--stats"],
    "fetch": ["--pmc", "FETCH_SIZE"],
    "write": ["--pmc", "WRITE_SIZE"],
    "req": ["--pmc", "TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"],
    "dram": ["--pmc", "TCC_BUBBLE_sum", "TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_RDREQ_DRAM_32B_sum", "TCC_MISS_sum"],
    "hit": ["--pmc", "TCC_HIT_sum", "TCC_REQ_sum", "TCC_READ_sum", "TCC_EA0_WRREQ_64B_sum"],
}


def run(out, prog):
    """Every pass of PASSES over the program, each under its own time limit; stops at a failure."""
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    for name, args in PASSES.items():
        print("pass", name, flush=True)
        with open(os.path.join(out, name + ".log"), "w") as log:
            subprocess.run(["timeout", "-s", "KILL", os.environ.get("PASS_TIMEOUT", "120"), "rocprofv3"] + args +
                           ["--output-format", "csv", "-d", os.path.join(out, name), "-o", name, "--"] + prog,
                           stdout=log, stderr=subprocess.STDOUT, env=env, check=True)
    print("passes done:", out)


def _rows(pattern):
    out = []
    for p in glob.glob(pattern):
        with open(p, newline="") as f:
            out += list(csv.DictReader(f))
    return out


def kernel_key(name: str) -> str:
    """Map a dispatch to its probe (kernel names: stream16, gather<F4, PIECE, TAG>)."""
    if "stream16" in name:
        return "stream16"
    if "gather<8" in name:
        return "gather128_dram"
    if "true" in name:
        return "gather16_dram"
    return "gather64_mall" if re.search(r"false, 0>", name) else "gather64_dram"


def summary(prof, out=None):
    known = {}
    for line in open(os.path.join(prof, "kt.log")):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            known[d["kernel"]] = d
    res = {}
    # kernel durations (second dispatch of each)
    disp = {}
    for sub in ("kt", "fetch", "write", "req", "dram", "hit"):
        for r in _rows(os.path.join(prof, sub, "*counter_collection.csv")) + \
                 _rows(os.path.join(prof, sub, "*kernel_trace.csv")):
            name = r.get("Kernel_Name", "")
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            disp.setdefault(sub, {}).setdefault(name, set()).add(did)
            if "Counter_Name" in r:
                res.setdefault(sub, []).append((did, name, r["Counter_Name"], float(r["Counter_Value"])))
            elif sub == "kt":
                res.setdefault("kt", []).append((did, name, "ns", float(r["End_Timestamp"]) - float(r["Start_Timestamp"])))
    table = {}
    for sub, rows in res.items():
        seen = {}
        for d, n, c, v in sorted(rows):
            seen.setdefault((kernel_key(n), c), []).append(v)
        for (key, c), vs in seen.items():
            table.setdefault(key, {})[c] = vs[-1]   # the second dispatch
    summary = {"source": "tools/hbm_probe.hip under tools/hbm_probe.py run (rocprofv3, one counter group per pass)",
               "kernels": {}}
    for key, d in known.items():
        t = table.get(key, {})
        b = float(d["bytes"])
        e = {"known_bytes": b, **({"table_bytes": d["table"]} if "table" in d else {}), "counters": t}
        if "FETCH_SIZE" in t:
            e["fetch_size_bytes"] = t["FETCH_SIZE"] * 1024
            e["fetch_size_over_known"] = e["fetch_size_bytes"] / b
        if "TCC_EA0_RDREQ_sum" in t:
            e["rdreq_x64_over_known"] = 64 * t["TCC_EA0_RDREQ_sum"] / b
            by = 32 * t.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * t.get("TCC_EA0_RDREQ_64B_sum", 0) + \
                128 * t.get("TCC_EA0_RDREQ_128B_sum", 0)
            e["rdreq_by_size_over_known"] = by / b
        if "TCC_EA0_RDREQ_DRAM_32B_sum" in t:
            e["dram_32b_x32_over_known"] = 32 * t["TCC_EA0_RDREQ_DRAM_32B_sum"] / b
        if "ns" in t:
            e["kernel_ms"] = t["ns"] / 1e6
            e["known_GBps"] = b / (t["ns"] * 1e-9) / 1e9
        summary["kernels"][key] = e
    path = out or os.path.join(ROOT, "profiles", "r03_hbm_probe.json")
    with open(path, "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        a = sys.argv[3:]
        run(sys.argv[2], a[1:] if a and a[0] == "--" else a)
    else:
        summary(*sys.argv[2:4])
