"""Per-launch SQ counter summary of rocprofv3 --pmc passes of the render kernel.

    python tools/summarize_sq.py DIR TAG [TAG ...]     (DIR/{a,b,c}_TAG/*_counter_collection.csv)
"""
import collections
import csv
import glob
import os
import sys


def load(d, tag, kernel="render_kernel"):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, f"*_{tag}", "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and "true" not in r["Kernel_Name"].split("<")[1][:12]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    ks = glob.glob(os.path.join(d, f"kt_{tag}", "*kernel_stats.csv"))
    if ks:
        for r in csv.DictReader(open(ks[0])):
            if kernel in r["Name"]:
                m["kernel_ms"] = float(r["AverageNs"]) / 1e6
    return m


def main():
    d = sys.argv[1]
    rows = {t: load(d, t) for t in sys.argv[2:]}
    keys = sorted(set().union(*[set(m) for m in rows.values()]))
    print("%-26s" % "counter" + "".join("%16s" % t for t in rows))
    for k in keys:
        print("%-26s" % k + "".join("%16.4g" % rows[t].get(k, float("nan")) for t in rows))
    for t, m in rows.items():
        wc = m.get("SQ_WAVE_CYCLES", 1)
        ins = sum(m.get(k, 0) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"))
        print(f"{t}: per wave-cycle issue {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} waitcnt {m.get('SQ_WAIT_ANY', 0) / wc:.3f} "
              f"stall {m.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}; instr/wave {ins / max(1, m.get('SQ_WAVES', 1)):.0f}; "
              f"VALU lanes active {m.get('SQ_THREAD_CYCLES_VALU', 0) / max(1, 64 * m.get('SQ_ACTIVE_INST_VALU', 1)):.3f}")


if __name__ == "__main__":
    main()
