"""Image parity metrics and the tolerance gate (TEST INFRASTRUCTURE ONLY).

Gate (BASELINE.md "Parity gate"), for two renders of the
same configuration with the same global pixel indexing:
  1. >= 99.5 % of pixels with per-pixel RGB L2 distance <= 1e-4
  2. image RMSE <= 0.01
  3. |channel mean difference| <= 1e-3 for each of R, G, B
The gate is meant for comparing against the reference implementation, whose
OpenCL builtins are implementation-defined; this package's GPU kernels and the
CPU oracle share the numerics contract and are compared bit for bit instead.
"""
from __future__ import annotations

import numpy as np

L2_TOL = 1e-4
FRAC_MIN = 0.995
RMSE_MAX = 0.01
MEAN_MAX = 1e-3


def stats(a, b) -> dict:
    a = np.asarray(a, np.float64).reshape(-1, 3)
    b = np.asarray(b, np.float64).reshape(-1, 3)
    assert a.shape == b.shape, (a.shape, b.shape)
    l2 = np.sqrt(((a - b) ** 2).sum(1))
    same = (np.asarray(a, np.float32) == np.asarray(b, np.float32)).all(1)
    return dict(
        pixels=int(a.shape[0]),
        frac_within=float((l2 <= L2_TOL).mean()) if a.size else 1.0,
        frac_identical=float(same.mean()) if a.size else 1.0,
        rmse=float(np.sqrt(((a - b) ** 2).mean())) if a.size else 0.0,
        max_l2=float(l2.max()) if a.size else 0.0,
        mean_diff=[float(x) for x in (a.mean(0) - b.mean(0))] if a.size else [0.0] * 3,
    )


def passes(st: dict) -> bool:
    return (st["frac_within"] >= FRAC_MIN and st["rmse"] <= RMSE_MAX
            and max(abs(x) for x in st["mean_diff"]) <= MEAN_MAX)


def assert_gate(a, b, what: str = "") -> dict:
    st = stats(a, b)
    assert passes(st), f"parity gate failed {what}: {st}"
    return st
