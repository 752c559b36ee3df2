"""Fixture from the reference's own committed render output/out.png (run where /root/reference exists).

out.png (== screenshots/Serre.png) is Serre_leger rendered by the reference at its .ini settings
(1024x1024, 100 spp, maxBounce 4) with the 8k IBL that is not in the repository, saved by
FileManager.saveImg as (x*255).astype(uint8).  We keep: the channel means of the whole image, the
512x512 centre crop, and 16x16 block means (64x64 thumbnail) -- enough for a loose end-to-end
check of the full kernel (the IBL substitute changes the background, so the comparison is loose).
"""
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("REFERENCE_ROOT", "/root/reference")
img = np.asarray(Image.open(os.path.join(REF, "output", "out.png")).convert("RGB"))
assert img.shape == (1024, 1024, 3), img.shape
c = img[256:768, 256:768]
thumb = img.reshape(64, 16, 64, 16, 3).mean((1, 3)).astype(np.float32)
np.savez_compressed(os.path.join(ROOT, "tests", "golden", "ref_outpng_serre.npz"), crop=c,
                    means=img.reshape(-1, 3).mean(0) / 255.0, thumb=thumb,
                    row_means=img.mean(1).astype(np.float32))
print("ok", img.reshape(-1, 3).mean(0) / 255.0)
