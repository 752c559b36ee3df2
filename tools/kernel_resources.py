"""Per-kernel register / scratch / LDS usage of the built HIP object (gfx950 code object notes), and
where the spill code sits.

    python tools/kernel_resources.py [build/native/rt_kernels.o] [name-filter]
    python tools/kernel_resources.py --loops OBJ MANGLED-NAME-PART
        every loop (backward branch) of that kernel's ISA with its scratch accesses, SGPR-spill lane
        moves (v_readlane / v_writelane), global loads and LDS operations: a traversal loop should show
        no scratch access
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(obj, td):
    fat = os.path.join(td, "fat.bin")
    co = os.path.join(td, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(td, "x.o")],
                   check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def loops(obj, pat):
    with tempfile.TemporaryDirectory() as td:
        co = code_object(obj, td)
        isa = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--symbolize-operands", co], capture_output=True,
                             text=True).stdout.split("\n")
    starts = [i for i, l in enumerate(isa) if re.match(r"^[0-9a-f]+ <_Z", l)] + [len(isa)]
    body = next((isa[a:b] for a, b in zip(starts, starts[1:]) if pat in isa[a]), None)
    if body is None:
        raise SystemExit(f"no kernel matching {pat!r}")
    print(body[0])
    labels = {m.group(1): k for k, x in enumerate(body) if (m := re.match(r"^[0-9a-f]+ <(L\d+)>:", x))}
    for k, x in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch) (L\d+)", x)
        if m and labels.get(m.group(1), k) < k:
            seg = body[labels[m.group(1)]:k + 1]
            cnt = lambda *ws: sum(any(w in y for w in ws) for y in seg)
            print(f"loop lines {labels[m.group(1)]}-{k}: scratch {cnt('scratch_')} lane-moves "
                  f"{cnt('v_readlane', 'v_writelane')} global_load {cnt('global_load')} lds {cnt('ds_read', 'ds_write')}")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--loops":
        return loops(sys.argv[2], sys.argv[3])
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "build", "native",
                                                              "rt_kernels.o")
    filt = sys.argv[2] if len(sys.argv) > 2 else "render"
    with tempfile.TemporaryDirectory() as td:
        co = code_object(obj, td)
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
