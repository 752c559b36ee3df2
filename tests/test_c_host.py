"""The boundary from a plain-C host (examples/render_scene.c): the headers compile as strict C11 and
C++17 against the in-tree library (CPU), and on the GPU the C program -- native OBJ import, native
BVH build, rt_scene_check, rt_render, rt_render_rgb8, rt_gamma -- renders exactly what the Python
KernelLauncher renders from the same inputs."""
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "ensem3a_openclraytracer_amd", "lib")
SRC = os.path.join(ROOT, "examples", "render_scene.c")
BIN = os.path.join(ROOT, "examples", "bin", "render_scene")


def test_example_compiles_and_links_as_strict_c(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libensem3a_rt.so")):
        pytest.skip("library not built")
    out = tmp_path / "render_scene"
    cmd = ["gcc", "-std=c11", "-pedantic", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
           SRC, "-L", LIBDIR, "-lensem3a_rt", "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, LD_LIBRARY_PATH=LIBDIR)
    run = subprocess.run([str(out)], capture_output=True, text=True, env=env)
    assert run.returncode == 2 and "usage" in run.stderr


@pytest.mark.parametrize("compiler", [["gcc", "-x", "c", "-std=c99", "-pedantic"], ["g++", "-x", "c++", "-std=c++17"]])
def test_every_header_compiles_as_c_and_cxx(tmp_path, compiler):
    """include/*.h in one translation unit, every declared entry point referenced, linked to the library."""
    if not os.path.exists(os.path.join(LIBDIR, "libensem3a_rt.so")):
        pytest.skip("library not built")
    from ensem3a_openclraytracer_amd import _native
    refs = "\n".join(f"    (void)&{name};" for name in sorted(_native.EXPORTED))
    tu = tmp_path / "headers.c"
    tu.write_text('#include "rt_api.h"\n#include "rt_debug.h"\n#include "rt_scene.h"\n'
                  f"int main(void) {{\n{refs}\n    return 0;\n}}\n")
    cmd = compiler + ["-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"), str(tu), "-x", "none",
                      "-L", LIBDIR, "-lensem3a_rt", "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(tmp_path / "h")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]


def _params(mat, cam, env, npix, spp, mb, ibl) -> bytes:
    h, w = ibl.shape[:2]
    mat = np.ascontiguousarray(mat, np.float32).reshape(-1)
    return (struct.pack("<i", mat.size // 6) + mat.tobytes() + np.asarray(cam, np.float32)[:10].tobytes()
            + np.asarray(env, np.float32)[:5].tobytes() + struct.pack("<iiiii", npix, spp, mb, w, h)
            + np.ascontiguousarray(ibl, np.uint8).tobytes())


@pytest.mark.gpu
@pytest.mark.parametrize("n,side,spp", [(24, 48, 4), (4, 32, 8)])
def test_c_host_renders_like_the_launcher(tmp_path, n, side, spp):
    """A grid heightfield (SURVEY.md Appendix D, 2 n^2 triangles, the default .ini template) rendered by
    the C program and by KernelLauncher: float frame, 8-bit frame and gamma output bit-identical."""
    from ensem3a_openclraytracer_amd import workloads as W
    from ensem3a_openclraytracer_amd.scene import Scene
    from ensem3a_openclraytracer_amd.KernelLauncher import KernelLauncher
    assert os.path.exists(BIN), "examples/bin/render_scene is built by __graft_entry__.build()"
    text = W.grid_obj_text(n)
    sc = Scene.from_text(text, None, build_bvh=True, name=f"grid{n}")
    cam, env = sc.camera(side, side), sc.env()
    npix, mb, ibl = side * side, 4, W.ibl_preview()
    (tmp_path / "grid.obj").write_text(text)
    (tmp_path / "params.bin").write_bytes(_params(sc.materialData, cam, env, npix, spp, mb, ibl))
    prefix = str(tmp_path / "out")
    r = subprocess.run([BIN, str(tmp_path / "grid.obj"), str(tmp_path / "params.bin"), prefix],
                       capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "refused as expected" in r.stdout
    got = np.fromfile(prefix + ".f32", np.float32)
    got8 = np.fromfile(prefix + ".rgb8", np.uint8)
    gotg = np.fromfile(prefix + ".gamma.f32", np.float32)

    kl = KernelLauncher(None, None, 0, None)
    try:
        want = np.zeros(3 * npix, np.float32)
        kl.launch_Raytracing(want, sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData,
                             sc.BVH.exportArray, cam, env, npix, spp, mb, ibl)
        want8 = np.zeros(3 * npix, np.uint8)
        kl.launch_Raytracing_rgb8(want8, sc.V_p, sc.V_n, sc.V_uv, sc.faceData, sc.materialData, sc.lightData,
                                  sc.BVH.exportArray, cam, env, npix, spp, mb, ibl)
        wantg = np.zeros(3 * npix, np.float32)
        kl.launch_ImgProcessing(want, wantg, side)   # the reference passes the image side (SIZE^2 pixels)
    finally:
        kl.close()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got8, want8)
    np.testing.assert_array_equal(gotg, wantg)
    assert want.mean() > 0.0
