import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def _ensure_built():
    from ensem3a_openclraytracer_amd import _build
    if not os.path.exists(_build.LIB):
        _build.build()
    from oracle import oracle as O
    if not os.path.exists(O._LIB_PATH):
        O.build()


_ensure_built()


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def kat_ref():
    import numpy as np
    p = os.path.join(GOLDEN, "kat_reference.npz")
    if not os.path.exists(p):
        pytest.skip("kat_reference.npz not generated yet (tools/gen_golden.py on the GPU box)")
    with np.load(p, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
