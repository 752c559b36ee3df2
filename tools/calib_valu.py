"""Converged reference kernel for counter calibration: 64M divisions (every lane active)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensem3a_openclraytracer_amd import _native
ctx = _native.Context()
x = np.random.default_rng(0).uniform(1, 2, 1 << 24).astype(np.float32)
for _ in range(3):
    ctx.debug_math(7, x, x)
print("ok")
