"""Host-side scene preparation: the flat arrays the path-tracing kernel reads.

This mirrors the data contract of the reference's ``FileManager.Scene``
(``FileManager.py:209-330``) and the packing done in ``main.main``
(``main.py:59-73``).  It is the caller side of the drop-in boundary: the
arrays produced here are exactly what ``KernelLauncher.launch_Raytracing``
receives in the reference, so a render driven from these arrays goes through
the same ``launch_Raytracing`` signature.

Layouts (all flat, little-endian, C-contiguous):

* ``V_p``  float32 [3*Nv]   vertex positions, OBJ ``v`` lines in file order
* ``V_n``  float32 [3*Nn]   vertex normals, OBJ ``vn`` lines
* ``V_uv`` float32 [2*Nt]   texture coordinates, OBJ ``vt`` lines
* ``faceData`` int32 [10*T] per triangle ``[mat, uv0,uv1,uv2, n0,n1,n2, p0,p1,p2]``
  (0-based indices, component order uv, n, p -- ``FileManager.py:276-282``)
* ``materialData`` float32 [6*M] per material ``[type, r, g, b, roughness, ior]``
  taken from the ``M_*`` keys of the scene ``.ini`` in file order
  (``FileManager.py:309-324``)
* ``lightData`` int32 [L]  indices of triangles whose material type is 0
  (``FileManager.py:234-240``)
* ``BVH.exportArray`` float32 [9*(2T-1)] built by :mod:`.bvh`.
"""
from __future__ import annotations

import io
import json
import os
from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

__all__ = [
    "parse_obj",
    "parse_ini",
    "material_array",
    "light_array",
    "pack_camera",
    "pack_env",
    "Scene",
    "DEFAULT_INI_TEMPLATE",
]

# Default .ini written by configReader when a scene has none (FileManager.py:356-383).
DEFAULT_INI_TEMPLATE = (
    "resolution=256\nspp=10\nmaxBounce=4\ncam_x=0\ncam_y=0\ncam_z=0\ncam_rx=0\n"
    "cam_ry=0\ncam_rz=0\ncam_DOF=45\nIBLfile=IBL/Arches_E_PineTree_8k.jpg\n"
    "IBL_Power=1.0\nsun_Power=1.0\nsun_rx=0\nsun_ry=0\nsun_rz=0\n"
)


def parse_obj(text: str):
    """Parse Wavefront OBJ text the way the reference importer does.

    Geometry (``v``/``vn``/``vt``) comes from every such line in file order
    (the reference reads them through pywavefront, ``FileManager.py:297-304``).
    Faces follow ``FileManager.py:265-291``:

    * lines before the first ``usemtl`` line are skipped (faces there are lost);
    * after it, every line whose first character is ``f`` is a triangle
      ``f p/uv/n p/uv/n p/uv/n`` (only the first three vertices are read);
    * every other line whose first character is ``u`` increments the current
      material index, which starts at 0 for the first ``usemtl``.

    Returns ``(V_p, V_n, V_uv, faceData, materialCount)`` where
    ``materialCount`` is the reference's ``matCounter`` (number of ``u`` lines
    after the first ``usemtl``).
    """
    vp, vn, vt = [], [], []
    faces = []
    mat_counter = 0
    seen_usemtl = False
    for raw in io.StringIO(text):
        line = raw
        toks = line.split()
        if toks:
            head = toks[0]
            if head == "v":
                vp.append((float(toks[1]), float(toks[2]), float(toks[3])))
            elif head == "vn":
                vn.append((float(toks[1]), float(toks[2]), float(toks[3])))
            elif head == "vt":
                u = float(toks[1])
                v = float(toks[2]) if len(toks) > 2 else 0.0
                vt.append((u, v))
        if not seen_usemtl:
            if line.split(" ")[0] == "usemtl":
                seen_usemtl = True
            continue
        if not line:
            continue
        if line[0] == "f":
            parts = line.split(" ")
            row = [mat_counter]
            for comp in (1, 2, 0):  # uv, normal, position (FileManager.py:279)
                for j in range(1, 4):
                    row.append(int(parts[j].split("/")[comp]) - 1)
            faces.append(row)
        elif line[0] == "u":
            mat_counter += 1
    V_p = np.asarray(vp, dtype=np.float64).astype(np.float32).reshape(-1)
    V_n = np.asarray(vn, dtype=np.float64).astype(np.float32).reshape(-1)
    V_uv = np.asarray(vt, dtype=np.float64).astype(np.float32).reshape(-1)
    faceData = np.asarray(faces, dtype=np.int32).reshape(-1)
    return V_p, V_n, V_uv, faceData, mat_counter


def parse_ini(text: str) -> Dict[str, str]:
    """``key=value`` lines into an insertion-ordered dict (``FileManager.py:399-408``).

    Duplicate keys keep their first position and last value, as a Python dict
    does in the reference.  Blank lines are skipped (the reference raises
    ``IndexError`` on them).
    """
    params: Dict[str, str] = {}
    for line in text.splitlines():
        if "=" not in line:
            if line.strip():
                raise ValueError(f"malformed .ini line {line!r}")
            continue
        parts = line.split("=")  # a value containing '=' keeps only its first field, as the reference
        params[parts[0]] = parts[1].split("\n")[0]
    return params


def material_array(params: Dict[str, str]) -> np.ndarray:
    """``materialData``: every ``M_*`` value in file order (``FileManager.py:314-323``)."""
    vals = [params[k] for k in params if k.split("_")[0] == "M"]
    return np.asarray([float(v) for v in vals], dtype=np.float64).astype(np.float32)


def light_array(faceData: np.ndarray, materialData: np.ndarray) -> np.ndarray:
    """Triangles whose material type is 0 (emissive), ``FileManager.py:234-240``."""
    face = np.asarray(faceData, dtype=np.int32).reshape(-1, 10)
    mats = np.asarray(materialData, dtype=np.float32)
    types = mats[face[:, 0] * 6]
    return np.nonzero(types == 0)[0].astype(np.int32)


def pack_camera(params: Dict[str, str], width: Optional[int] = None,
                height: Optional[int] = None) -> np.ndarray:
    """``cam float32[10]`` exactly as ``main.py:59-61`` packs it.

    ``[x, y, z, rx, ry, rz, resX, resY, 1, DOF*(3.14/180)]``; the field of view
    is multiplied in float64 then cast to float32, like the reference.
    """
    res = int(params["resolution"])
    w = res if width is None else int(width)
    h = res if height is None else int(height)
    return np.array([
        float(params["cam_x"]), float(params["cam_y"]), float(params["cam_z"]),
        float(params["cam_rx"]), float(params["cam_ry"]), float(params["cam_rz"]),
        w, h, 1, float(params["cam_DOF"]) * (3.14 / 180)], dtype=np.float64).astype(np.float32)


def pack_env(params: Dict[str, str]) -> np.ndarray:
    """``envData float32[5] = [sun_rx, sun_ry, sun_rz, sun_Power, IBL_Power]`` (``main.py:72-73``)."""
    return np.array([float(params["sun_rx"]), float(params["sun_ry"]), float(params["sun_rz"]),
                     float(params["sun_Power"]), float(params["IBL_Power"])],
                    dtype=np.float64).astype(np.float32)


@dataclass
class _BVHHolder:
    """Stands where the reference keeps ``scene.BVH`` (only ``exportArray`` is read, ``main.py:85``)."""
    exportArray: np.ndarray


@dataclass
class Scene:
    """The arrays of ``FileManager.Scene`` plus its parameters.

    Construct with :meth:`from_obj` (OBJ + ``.ini`` text, or paths) or
    :meth:`load` (a packed ``.npz`` produced by :meth:`save`).
    """
    V_p: np.ndarray
    V_n: np.ndarray
    V_uv: np.ndarray
    faceData: np.ndarray
    materialData: np.ndarray
    lightData: np.ndarray
    params: Dict[str, str] = field(default_factory=dict)
    materialCount: int = 0
    name: str = ""
    _bvh: Optional[_BVHHolder] = None

    # -- construction -------------------------------------------------
    @classmethod
    def from_obj(cls, obj_path: str, ini_path: Optional[str] = None, build_bvh: bool = True,
                 name: Optional[str] = None) -> "Scene":
        with open(obj_path, "r") as f:
            obj_text = f.read()
        if ini_path is None:
            ini_path = obj_path.replace(".obj", ".ini")
        if os.path.exists(ini_path):
            with open(ini_path, "r") as f:
                ini_text = f.read()
        else:
            ini_text = None
        return cls.from_text(obj_text, ini_text, build_bvh=build_bvh,
                             name=name or os.path.splitext(os.path.basename(obj_path))[0])

    @classmethod
    def from_text(cls, obj_text: str, ini_text: Optional[str], build_bvh: bool = True,
                  name: str = "") -> "Scene":
        # the native importer (csrc/obj_load.cpp) is the same parse, ~50x faster on 1M-triangle files
        from . import _native
        V_p, V_n, V_uv, faceData, mat_count = _native.parse_obj(obj_text)
        if ini_text is None:
            # configReader default fill (FileManager.py:356-383): materialCount+1 white diffuse
            ini_text = DEFAULT_INI_TEMPLATE + "".join(
                f"M_{i}_Type=1\nM_{i}_Color_R=1\nM_{i}_Color_G=1\nM_{i}_Color_B=1\n"
                f"M_{i}_roughness=0\nM_{i}_ior=0\n" for i in range(mat_count + 1))
        params = parse_ini(ini_text)
        materialData = material_array(params)
        lightData = light_array(faceData, materialData) if faceData.size else np.zeros(0, np.int32)
        sc = cls(V_p, V_n, V_uv, faceData, materialData, lightData, params, mat_count, name)
        if build_bvh:
            sc.build_bvh()
        return sc

    # -- BVH ------------------------------------------------------------
    def build_bvh(self) -> np.ndarray:
        from .bvh import build_export_array
        self._bvh = _BVHHolder(build_export_array(self.faceData, self.V_p))
        return self._bvh.exportArray

    @property
    def BVH(self) -> _BVHHolder:
        if self._bvh is None:
            self.build_bvh()
        return self._bvh

    @property
    def triCount(self) -> int:
        return int(self.faceData.size // 10)

    # -- parameters -----------------------------------------------------
    def loadParameters(self) -> Dict[str, str]:
        return dict(self.params)

    def set_material(self, index: int, type_: Optional[float] = None, color=None,
                     roughness: Optional[float] = None) -> None:
        """Override material ``index`` (used by the bench configs, e.g. C3's glass monkey)."""
        base = 6 * index
        if type_ is not None:
            self.params[f"M_{index}_Type"] = repr(type_)
        if color is not None:
            for c, key in zip(color, ("Color_R", "Color_G", "Color_B")):
                self.params[f"M_{index}_{key}"] = repr(float(c))
        if roughness is not None:
            self.params[f"M_{index}_roughness"] = repr(float(roughness))
        self.materialData = material_array(self.params)
        assert self.materialData.size > base
        self.lightData = light_array(self.faceData, self.materialData)

    def camera(self, width: Optional[int] = None, height: Optional[int] = None) -> np.ndarray:
        return pack_camera(self.params, width, height)

    def env(self) -> np.ndarray:
        return pack_env(self.params)

    # -- persistence ----------------------------------------------------
    def save(self, path: str, with_bvh: bool = False) -> None:
        arrays = dict(V_p=self.V_p, V_n=self.V_n, V_uv=self.V_uv, faceData=self.faceData,
                      materialData=self.materialData, lightData=self.lightData,
                      params=np.frombuffer(json.dumps(self.params).encode(), dtype=np.uint8),
                      meta=np.array([self.materialCount], dtype=np.int64))
        if with_bvh:
            arrays["BVH"] = self.BVH.exportArray
        np.savez_compressed(path, **arrays)

    @classmethod
    def load(cls, path: str, build_bvh: bool = True) -> "Scene":
        with np.load(path, allow_pickle=False) as z:
            params = json.loads(bytes(z["params"]).decode())
            sc = cls(z["V_p"].copy(), z["V_n"].copy(), z["V_uv"].copy(), z["faceData"].copy(),
                     z["materialData"].copy(), z["lightData"].copy(), params,
                     int(z["meta"][0]), os.path.splitext(os.path.basename(path))[0])
            if "BVH" in z.files:
                sc._bvh = _BVHHolder(z["BVH"].copy())
        if build_bvh and sc._bvh is None:
            sc.build_bvh()
        return sc
