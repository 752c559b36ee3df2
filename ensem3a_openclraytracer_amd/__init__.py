"""MI355X-native path-tracing integrator (drop-in for the reference's OpenCL path).

Public surface:
  * :class:`KernelLauncher` -- the reference's ``KernelLauncher`` API backed by
    HIP kernels for gfx950 through a ctypes C-ABI (include/rt_api.h);
  * :class:`Scene` / :func:`bvh.build_export_array` -- the host data contract
    (``FileManager.Scene`` arrays, ``BVH.exportArray``);
  * :mod:`.render` -- ``main.main``-equivalent render driver and multi-GPU tiling.
"""
from .scene import Scene, pack_camera, pack_env  # noqa: F401

__all__ = ["Scene", "pack_camera", "pack_env", "KernelLauncher"]


def __getattr__(name):
    if name == "KernelLauncher":
        from .KernelLauncher import KernelLauncher
        return KernelLauncher
    raise AttributeError(name)
