"""Pack the reference's bundled scenes into in-repo inputs (run where /root/reference exists).

Writes ensem3a_openclraytracer_amd/scenes/<name>.npz (V_p, V_n, V_uv, faceData,
materialData, lightData and the .ini parameters, produced by this package's own
OBJ/.ini loader, scene.py) and ibl_preview.npz (the bundled 600x300 IBL preview,
decoded to RGBA8 with PIL exactly as main.py:68 converts the IBL).  These are the
benchmark/parity inputs that travel to the GPU box.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ensem3a_openclraytracer_amd.scene import Scene  # noqa: E402

REF = os.environ.get("REFERENCE_ROOT", "/root/reference")
OUT = os.path.join(ROOT, "ensem3a_openclraytracer_amd", "scenes")
NAMES = {"Cornell box": "cornell", "Cornell box_Monkey": "monkey", "Serre_leger": "serre",
         "protoEnsem": "proto", "FurnaceHD": "furnace"}


def main():
    os.makedirs(OUT, exist_ok=True)
    for src, dst in NAMES.items():
        sc = Scene.from_obj(os.path.join(REF, "ObjFiles", src + ".obj"), build_bvh=False)
        sc.save(os.path.join(OUT, dst + ".npz"))
        print(dst, sc.triCount, "tris")
    from PIL import Image
    img = Image.open(os.path.join(REF, "IBL", "Arches_E_PineTree_Preview.jpg")).convert("RGBA")
    rgba = np.frombuffer(img.tobytes(), dtype=np.uint8).reshape(img.size[1], img.size[0], 4)
    np.savez_compressed(os.path.join(OUT, "ibl_preview.npz"), rgba=rgba)
    print("ibl", rgba.shape)


if __name__ == "__main__":
    main()
