"""The benchmark configurations of BASELINE.json and small parity cases.

Each :class:`Workload` resolves to exactly the arguments the reference's
``launch_Raytracing`` receives (scene arrays, ``cam[10]``, ``envData[5]``,
``imgDim``, ``spp``, ``maxBounce``, IBL texels).

* C1 ``cornell_256_s4``  -- Cornell box 256x256, 4 spp (the reference's CPU case)
* C2 ``cornell_1024_s64`` -- Cornell box 1024x1024, 64 spp, diffuse only (headline)
* C3 ``monkey_1024_s256`` -- Monkey box 1024x1024, 256 spp, glass monkey + glossy walls
* C4 ``serre_1920x1080_s512`` -- Serre_leger 1920x1080, 512 spp, 8k IBL substitute
* C5 ``grid1m_3840x2160_s1024`` -- synthetic 1M-triangle grid
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from functools import lru_cache
from typing import Dict, Optional, Tuple

import numpy as np

from .scene import Scene

SCENE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "scenes")
MAX_BOUNCE = 4  # every bundled .ini (e.g. ObjFiles/Cornell box.ini:4)


@lru_cache(maxsize=None)
def ibl_preview() -> np.ndarray:
    """The bundled 600x300 IBL preview as RGBA8 (HxWx4)."""
    with np.load(os.path.join(SCENE_DIR, "ibl_preview.npz"), allow_pickle=False) as z:
        return z["rgba"].copy()


@lru_cache(maxsize=None)
def ibl_8k() -> np.ndarray:
    """8192x4096 RGBA8 substitute for the missing Arches_E_PineTree_8k.jpg (main.py:68):
    PIL bilinear upscale of the preview."""
    from PIL import Image
    prev = ibl_preview()
    img = Image.fromarray(prev, "RGBA").resize((8192, 4096), Image.BILINEAR)
    return np.frombuffer(img.tobytes(), dtype=np.uint8).reshape(4096, 8192, 4).copy()


def load_scene(name: str) -> Scene:
    return Scene.load(os.path.join(SCENE_DIR, name + ".npz"))


def grid_obj_text(n: int = 708) -> str:
    """SURVEY.md Appendix D synthetic heightfield: 2*n^2 triangles, (n+1)^2 vertices."""
    x = np.linspace(-1.0, 1.0, n + 1)
    z = np.linspace(-1.0, 1.0, n + 1)
    X, Z = np.meshgrid(x, z, indexing="ij")
    noise = np.random.default_rng(0).standard_normal((n + 1, n + 1))
    Y = 2.0 + 0.05 * np.sin(9.0 * X) * np.cos(7.0 * Z) + 0.01 * noise
    lines = ["o grid"]
    lines += ["v %.6f %.6f %.6f" % (a, b, c) for a, b, c in zip(X.ravel(), Y.ravel(), Z.ravel())]
    lines += ["vt 0 0", "vn 0 -1 0", "usemtl White", "s off"]
    idx = lambda i, j: i * (n + 1) + j + 1  # noqa: E731
    for i in range(n):
        for j in range(n):
            a, b, c, d = idx(i, j), idx(i + 1, j), idx(i + 1, j + 1), idx(i, j + 1)
            lines.append(f"f {a}/1/1 {b}/1/1 {c}/1/1")
            lines.append(f"f {a}/1/1 {c}/1/1 {d}/1/1")
    return "\n".join(lines) + "\n"


@lru_cache(maxsize=None)
def grid_scene(n: int = 708) -> Scene:
    return Scene.from_text(grid_obj_text(n), None, build_bvh=True, name=f"grid{n}")


@dataclass
class Workload:
    name: str
    scene: str
    width: int
    height: int
    spp: int
    max_bounce: int = MAX_BOUNCE
    overrides: Tuple = ()          # (material index, type, color, roughness)
    ibl: str = "preview"           # "preview" or "8k"
    params: Dict[str, str] = field(default_factory=dict)  # .ini overrides (camera/env)

    @property
    def npix(self) -> int:
        return self.width * self.height

    @property
    def samples(self) -> int:
        return self.npix * self.spp

    def build_scene(self) -> Scene:
        sc = grid_scene() if self.scene == "grid1m" else load_scene(self.scene)
        for m, t, col, rough in self.overrides:
            sc.set_material(m, type_=t, color=col, roughness=rough)
        sc.params.update(self.params)
        return sc

    def data_note(self) -> str:
        src = {"cornell": "ObjFiles/Cornell box.obj + .ini", "monkey": "ObjFiles/Cornell box_Monkey.obj + .ini",
               "serre": "ObjFiles/Serre_leger.obj + .ini", "proto": "ObjFiles/protoEnsem.obj + .ini",
               "furnace": "ObjFiles/FurnaceHD.obj + .ini",
               "grid1m": "synthetic 1M-triangle grid (SURVEY.md Appendix D)"}.get(self.scene, self.scene)
        note = f"reference scene {src}" if self.scene != "grid1m" else src
        if self.overrides:
            note += " with the config's material overrides"
        ibl = "8k IBL substitute (bilinear upscale of the bundled preview)" if self.ibl == "8k" else "bundled preview IBL"
        return f"{note}, {ibl}; scene and IBL resident in HBM"

    def ibl_rgba(self) -> np.ndarray:
        return ibl_8k() if self.ibl == "8k" else ibl_preview()

    def inputs(self, scene: Optional[Scene] = None):
        """(scene, cam, env, npix, spp, max_bounce, ibl) for launch_Raytracing."""
        sc = scene or self.build_scene()
        cam = sc.camera(self.width, self.height)
        return sc, cam, sc.env(), self.npix, self.spp, self.max_bounce, self.ibl_rgba()

    def with_size(self, width: int, height: int, spp: Optional[int] = None) -> "Workload":
        return Workload(self.name + f"@{width}x{height}s{spp or self.spp}", self.scene, width, height,
                        spp or self.spp, self.max_bounce, self.overrides, self.ibl, dict(self.params))


C3_OVERRIDES = ((4, 3.0, (0.88, 1.0, 1.0), None), (0, 2.0, None, 0.2))

CONFIGS: Dict[str, Workload] = {
    "C1": Workload("cornell_256_s4", "cornell", 256, 256, 4),
    "C2": Workload("cornell_1024_s64", "cornell", 1024, 1024, 64),
    "C3": Workload("monkey_1024_s256", "monkey", 1024, 1024, 256, overrides=C3_OVERRIDES),
    "C4": Workload("serre_1920x1080_s512", "serre", 1920, 1080, 512, ibl="8k"),
    "C5": Workload("grid1m_3840x2160_s1024", "grid1m", 3840, 2160, 1024, ibl="8k"),
}

# Small cases the CPU oracle finishes in seconds (parity fixtures).
PARITY_CASES: Dict[str, Workload] = {
    "cornell_64_s4": Workload("cornell_64_s4", "cornell", 64, 64, 4),
    "cornell_128_s16": Workload("cornell_128_s16", "cornell", 128, 128, 16),
    "cornell_64_b0": Workload("cornell_64_b0", "cornell", 64, 64, 3, max_bounce=0),
    "cornell_32_s0": Workload("cornell_32_s0", "cornell", 32, 32, 0),
    "monkey_c3_64_s4": Workload("monkey_c3_64_s4", "monkey", 64, 64, 4, overrides=C3_OVERRIDES),
    "monkey_ini_64_s4": Workload("monkey_ini_64_s4", "monkey", 64, 64, 4),
    "serre_96x54_s4": Workload("serre_96x54_s4", "serre", 96, 54, 4),
    "proto_64_s4": Workload("proto_64_s4", "proto", 64, 64, 4),
    "furnace_64_s4": Workload("furnace_64_s4", "furnace", 64, 64, 4),
}
