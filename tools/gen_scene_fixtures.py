"""Scene-array fixtures from the reference's own importer (run where /root/reference exists).

    python tools/gen_scene_fixtures.py  ->  tests/golden/ref_scene_arrays.json

For every bundled scene with an .ini, the reference's ``FileManager.Scene(path, False, None)``
(FileManager.py:209-324) is constructed from /root/reference and its arrays are recorded:
``faceData`` (uv, n, p component order, the ``u``-line material counting, faces only after the
first ``usemtl``), ``materialData`` (the ``M_*`` keys in .ini order), ``lightData`` and the vertex
arrays, as sha256 digests (plus the small arrays in full).  ``cam``/``envData`` are packed from the
reference's own ``loadParameters()`` with the expressions of main.py:59-61 and 72-73 (main.py
itself imports pyopencl, which is absent, so it cannot be imported).

Two dependencies of FileManager.py are absent from this image:
  * pywavefront (unpinned: the reference has no requirements file).  FileManager reads only
    ``Wavefront(...).vertices``, ``.parser.normals``, ``.parser.tex_coords`` and ``.materials``
    (FileManager.py:260-304), i.e. the ``v``/``vn``/``vt`` lines as float tuples; the stand-in
    below supplies exactly that, so V_p/V_n/V_uv are pinned as far as that parse is;
  * nothing else: numpy, PIL, matplotlib and the reference's BVH.py import as they are.
The reference tree is read-only: bytecode writing is disabled and no .ini is created (scenes
without one are skipped).  Nothing from the reference is copied: the output is digests and
the small arrays.
"""
import hashlib
import json
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("REFERENCE_ROOT", "/root/reference")
OUT = os.path.join(ROOT, "tests", "golden", "ref_scene_arrays.json")
SCENES = {"Cornell box": "cornell", "Cornell box_Monkey": "monkey", "Serre_leger": "serre",
          "protoEnsem": "proto", "FurnaceHD": "furnace"}


def _pywavefront_standin():
    """The attributes of pywavefront.Wavefront that FileManager.py:260-304 reads."""
    mod = types.ModuleType("pywavefront")

    class Wavefront:
        def __init__(self, path, collect_faces=False, create_materials=True, **_):
            self.vertices, normals, tex = [], [], []
            with open(path) as f:
                for line in f:
                    t = line.split()
                    if not t:
                        continue
                    if t[0] == "v":
                        self.vertices.append(tuple(float(x) for x in t[1:4]))
                    elif t[0] == "vn":
                        normals.append(tuple(float(x) for x in t[1:4]))
                    elif t[0] == "vt":
                        tex.append((float(t[1]), float(t[2]) if len(t) > 2 else 0.0))
            self.parser = types.SimpleNamespace(normals=normals, tex_coords=tex)
            self.materials = {}

    mod.Wavefront = Wavefront
    return mod


def digest(a: np.ndarray) -> dict:
    a = np.ascontiguousarray(a)
    return {"dtype": str(a.dtype), "size": int(a.size), "sha256": hashlib.sha256(a.tobytes()).hexdigest()}


def main():
    sys.dont_write_bytecode = True
    sys.modules["pywavefront"] = _pywavefront_standin()
    sys.path.insert(0, REF)
    import FileManager  # the reference's importer
    out = {"generator": "tools/gen_scene_fixtures.py", "source": "FileManager.Scene (FileManager.py:209-324), "
           "cam/envData packed as main.py:59-61, 72-73", "scenes": {}}
    devnull = open(os.devnull, "w")
    for src, name in SCENES.items():
        obj = os.path.join(REF, "ObjFiles", src + ".obj")
        if not os.path.exists(obj.replace(".obj", ".ini")):
            continue
        stdout, sys.stdout = sys.stdout, devnull    # the importer prints progress
        try:
            sc = FileManager.Scene(obj, False, None)
        finally:
            sys.stdout = stdout
        p = sc.loadParameters()
        res = int(p["resolution"])
        cam = np.array([float(p["cam_x"]), float(p["cam_y"]), float(p["cam_z"]),
                        float(p["cam_rx"]), float(p["cam_ry"]), float(p["cam_rz"]),
                        res, res, 1, float(p["cam_DOF"]) * (3.14 / 180)]).astype(np.float32)
        env = np.array([float(p["sun_rx"]), float(p["sun_ry"]), float(p["sun_rz"]),
                        float(p["sun_Power"]), float(p["IBL_Power"])]).astype(np.float32)
        rec = {k: digest(getattr(sc, k)) for k in ("V_p", "V_n", "V_uv", "faceData", "materialData", "lightData")}
        rec["materialData"]["values"] = [float(x) for x in sc.materialData]
        rec["lightData"]["values"] = [int(x) for x in sc.lightData][:4096]
        rec["materialCount"] = int(sc.materialCount)
        rec["cam"] = [float(x) for x in cam]
        rec["env"] = [float(x) for x in env]
        rec["cam_bits"] = [int(x) for x in cam.view(np.uint32)]
        rec["env_bits"] = [int(x) for x in env.view(np.uint32)]
        out["scenes"][name] = rec
        print(name, sc.faceData.size // 10, "triangles")
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
