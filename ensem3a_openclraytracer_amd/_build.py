"""Build the native library (HIP kernels for gfx950 + the C-ABI) in-tree.

``python -m ensem3a_openclraytracer_amd._build`` or ``__graft_entry__.build()``.
Output: ``ensem3a_openclraytracer_amd/lib/libensem3a_rt.so``.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libensem3a_rt.so")
OBJDIR = os.path.join(ROOT, "build", "native")

SOURCES = ["rt_kernels.hip", "rt_spec.hip", "rt_api.hip", "scene_pack.cpp", "bvh_build.cpp", "bvh_sah.cpp", "obj_load.cpp"]
HEADERS = ["rt_internal.h", "rt_layout.h", "scene_pack.h", "rt_device.h", "rtm.h", "bvh_sah.h"]
# -ffp-contract=off: the numerics contract (rtm.h) places every fused multiply-add explicitly.
COMMON = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize", "-fPIC", "-Wall",
          "-Wno-unused-function", "-I", os.path.join(ROOT, "include")]


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build the native library")


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, force: bool = False, defines=(), out: str = None) -> str:
    """Compile the library; ``defines``/``out`` build an experimental variant elsewhere."""
    hipcc = _hipcc()
    lib_path = out or LIB
    objdir = OBJDIR if not defines else os.path.join(OBJDIR, "v_" + "_".join(d.replace("=", "") for d in defines))
    os.makedirs(objdir, exist_ok=True)
    os.makedirs(os.path.dirname(lib_path), exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", h)
                                                      for h in ("rt_api.h", "rt_debug.h", "rt_scene.h")]
    jobs = []
    objs = []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        if force or _newer(obj, [path] + hdrs):
            cmd = [hipcc] + COMMON + ["-D" + d for d in defines]
            if src.endswith(".hip"):
                cmd += ["--offload-arch=gfx950", "-x", "hip"]
            cmd += ["-c", path, "-o", obj]
            jobs.append(cmd)

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    if force or jobs or _newer(lib_path, objs):
        run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", "-o", lib_path] + objs)
    return lib_path


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
