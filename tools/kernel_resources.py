"""Per-kernel register / scratch / LDS usage of the built HIP object (gfx950 code object notes).

    python tools/kernel_resources.py [build/native/rt_kernels.o] [name-filter]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "build", "native",
                                                              "rt_kernels.o")
    filt = sys.argv[2] if len(sys.argv) > 2 else "render"
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        co = os.path.join(td, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(td, "x.o")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    cur = {}
    rows = []
    for line in notes.splitlines():
        m = re.match(r"\s*\.(name|private_segment_fixed_size|vgpr_count|sgpr_count|group_segment_fixed_size|"
                     r"vgpr_spill_count|sgpr_spill_count|agpr_count):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "name" and not v.endswith(".kd"):
            if cur.get("name"):
                rows.append(cur)
            cur = {"name": v}
        elif cur:
            cur[k] = v
    if cur.get("name"):
        rows.append(cur)
    for r in rows:
        if filt in r["name"]:
            print(f"vgpr {r.get('vgpr_count', '?'):>4} agpr {r.get('agpr_count', '?'):>3} sgpr {r.get('sgpr_count', '?'):>4} "
                  f"scratch {r.get('private_segment_fixed_size', '?'):>5} spill v/s {r.get('vgpr_spill_count', '?')}/"
                  f"{r.get('sgpr_spill_count', '?')}  {r['name']}")


if __name__ == "__main__":
    main()
