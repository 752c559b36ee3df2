"""Print per-launch PMC values of the render kernel from tools/run_diag.sh output."""
import csv, glob, re, sys, collections
import numpy as np
prof = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else r"render(_resume)?_kernel<(0, )?false, false"
vals = collections.defaultdict(list)
for p in glob.glob(prof + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(p, newline="")):
        if re.search(kern, r["Kernel_Name"]):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
v = {k: float(np.mean(x)) for k, x in vals.items()}
for k in sorted(v):
    print(f"{k:32s} {v[k]:.6g}")
def g(k): return v.get(k, float("nan"))
print("--- derived")
print("VALU lane utilisation  ", g("SQ_THREAD_CYCLES_VALU") / max(1, g("SQ_ACTIVE_INST_VALU")) / 64)
print("wait fraction          ", g("SQ_WAIT_ANY") / max(1, g("SQ_WAVE_CYCLES")))
print("issue-stall fraction   ", g("SQ_WAIT_INST_ANY") / max(1, g("SQ_WAVE_CYCLES")))
print("active fraction        ", g("SQ_ACTIVE_INST_ANY") / max(1, g("SQ_WAVE_CYCLES")))
print("VALU insts per wave    ", g("SQ_INSTS_VALU") / max(1, g("SQ_WAVES")))
print("VMEM rd insts per wave ", g("SQ_INSTS_VMEM_RD") / max(1, g("SQ_WAVES")))
print("avg waves resident/CU  ", g("SQ_WAVE_CYCLES") * 4 / max(1, g("SQ_BUSY_CYCLES")) / 256 if "SQ_BUSY_CYCLES" in v else None)
