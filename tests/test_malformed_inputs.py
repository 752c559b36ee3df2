"""Malformed and hostile scene input through the host-only native entry points (no GPU): the OBJ
importer (rt_obj_parse, FileManager.py:253-307), the BVH.py-exact builder (rt_bvh_build,
BVH.py:120-191) and the scene validation + repacking rt_set_scene applies (rt_scene_check,
KernelLauncher.py:38-72's buffers).  The reference either raises (Python int()/float() on a bad
field), indexes out of range, or loops forever (a cyclic or degenerate BVH); the native code must
refuse each case with an error, never read out of bounds or hang.

tools/sanitize.sh runs this file (and the rest of the CPU suite) against the ASan/UBSan build of
the same sources (oracle/Makefile asan, _native.HOST_ONLY)."""
import math

import numpy as np
import pytest

from ensem3a_openclraytracer_amd import _native
from ensem3a_openclraytracer_amd import bvh as B
from ensem3a_openclraytracer_amd import workloads as W

RT_ERR_ARG, RT_ERR_SCENE = 1, 4

TRI = "v 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nvt 0 0\nusemtl m\n"


# ---- OBJ text ----

@pytest.mark.parametrize("text", [
    TRI + "f",                                  # face keyword alone
    TRI + "f 1/1/1",                            # truncated after one vertex
    TRI + "f 1/1/1 2/1/1",                      # truncated after two vertices
    TRI + "f 1/1/1 2/1/1 3/1",                  # third vertex without its normal
    TRI + "f 1/1/1 2/1/1 /1/1\n",               # empty position field
    TRI + "f 1/1/1 2/1/1 3/x/1\n",              # non-numeric index
    TRI + "f 1/1/1 2/1/1 3/1/99999999999999999999999999\n",   # beyond int32 (and int64)
    TRI + "f 1/1/1 2/1/1 -9999999999/1/1\n",    # below int32
    "v 1 2\n",                                  # short vertex
    "v 1 2 x\n",                                # non-numeric coordinate
    "vn 1 2 3e\n",
    "vt\n",
])
def test_obj_parse_refuses_malformed_lines(text):
    with pytest.raises(ValueError):
        _native.parse_obj(text)


def test_obj_parse_odd_but_valid_text():
    # NUL bytes, CR line ends, a huge line, non-finite coordinates, no trailing newline: parsed as the
    # reference's float() / split() read them, without reading past the buffer
    text = "v nan inf -inf\nv 1e400 -1e400 1e-400\r\nvn 0 0 1\n# " + "x" * 100000 + "\n\x00\x01\nusemtl a\n" \
           "f 1/1/1 2/1/1 2/1/1"
    vp, vn, vuv, face, nmat = _native.parse_obj(text)
    assert math.isnan(vp[0]) and vp[1] == np.inf and vp[2] == -np.inf
    assert vp[3] == np.inf and vp[4] == -np.inf and vp[5] == 0.0
    assert face.tolist() == [0, 0, 0, 0, 0, 0, 0, 0, 1, 1]
    assert _native.parse_obj("")[3].size == 0
    assert _native.parse_obj(b"\xff\xfe\x00" * 1000)[3].size == 0


def test_obj_parse_keeps_out_of_range_indices_for_the_builder():
    # the reference's parse does no range check (FileManager.py:276-282); the index is caught downstream
    vp, vn, vuv, face, _ = _native.parse_obj(TRI + "f 1/1/1 2/1/1 7/1/1\n")
    assert face[9] == 6
    with pytest.raises(ValueError, match="out of range"):
        B.build_export_array(face, vp)
    with pytest.raises(_native.NativeError) as e:
        _native.scene_check(vp, vn, face, np.array([1, 1, 1, 1, 0, 0], np.float32), np.zeros(9, np.float32))
    assert e.value.status == RT_ERR_ARG


# ---- BVH builder ----

def test_bvh_build_refuses_degenerate_and_non_finite_input():
    face = np.array([0, 0, 0, 0, 0, 0, 0, 0, 1, 2] * 2, np.int32)   # the same triangle twice
    vp = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0], np.float32)
    with pytest.raises(B.DegenerateBVHError):
        B.build_export_array(face, vp)
    # a NaN vertex makes every centroid comparison false: one side of the split is empty
    face2 = np.array([0, 0, 0, 0, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 0, 0, 0, 3, 4, 5], np.int32)
    vp2 = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0, np.nan, 5, 5, 6, 5, 5, 5, 6, 5], np.float32)
    with pytest.raises(B.DegenerateBVHError):
        B.build_export_array(face2, vp2)
    # negative index
    with pytest.raises(ValueError, match="out of range"):
        B.build_export_array(np.array([0, 0, 0, 0, 0, 0, 0, -1, 1, 2], np.int32), vp)
    with pytest.raises(ValueError):
        B.build_export_array(np.zeros(7, np.int32), vp)   # truncated faceData


def test_bvh_build_infinite_vertices_terminates():
    # inf coordinates give inf / NaN centroids: either a tree over all triangles or the degenerate error
    face = np.array([[0, 0, 0, 0, 0, 0, 0, 3 * t, 3 * t + 1, 3 * t + 2] for t in range(4)], np.int32).ravel()
    vp = np.arange(36, dtype=np.float32)
    vp[5] = np.inf
    vp[20] = -np.inf
    try:
        out = B.build_export_array(face, vp)
    except B.DegenerateBVHError:
        return
    assert out.size == 9 * 7


# ---- scene validation (rt_set_scene's checks, host only) ----

def _cornell():
    sc, *_ = W.CONFIGS["C1"].inputs()
    return sc


def test_scene_check_accepts_the_bundled_scene():
    sc = _cornell()
    info = _native.scene_check(sc.V_p, sc.V_n, sc.faceData, sc.materialData, sc.BVH.exportArray)
    assert info["fast_ok"] and info["tris"] == 36 and info["brute_records"] == 36 and info["brute_boxes"] == 22
    ref = _native.scene_check(sc.V_p, sc.V_n, sc.faceData, sc.materialData, sc.BVH.exportArray,
                              layout=_native.RT_BVH_REFERENCE)
    assert ref["nodes"] == 35


def _expect(status, V_p, V_n, face, mat, bvh, match=None):
    with pytest.raises(_native.NativeError, match=match) as e:
        _native.scene_check(V_p, V_n, face, mat, bvh)
    assert e.value.status == status


def test_scene_check_refuses_bad_arrays():
    sc = _cornell()
    vp, vn, face, mat, bvh = sc.V_p, sc.V_n, sc.faceData, sc.materialData, sc.BVH.exportArray
    _expect(RT_ERR_ARG, vp[:-1], vn, face, mat, bvh, "sizes")            # truncated V_p
    _expect(RT_ERR_ARG, vp, vn, face[:-3], mat, bvh, "sizes")            # truncated faceData
    _expect(RT_ERR_ARG, vp, vn, face, mat[:-1], bvh, "sizes")            # truncated materialData
    _expect(RT_ERR_ARG, vp, vn, face, mat, bvh[:-4], "sizes")            # truncated BVH
    _expect(RT_ERR_SCENE, vp, vn, face, mat, bvh[:0], "without a BVH")
    bad = face.copy(); bad[17] = vp.size // 3                            # position index = vertex count
    _expect(RT_ERR_ARG, vp, vn, bad, mat, bvh, "position index")
    bad = face.copy(); bad[4] = -5                                       # negative normal index
    _expect(RT_ERR_ARG, vp, vn, bad, mat, bvh, "normal index")
    bad = face.copy(); bad[0] = 1 << 30                                  # material index
    _expect(RT_ERR_ARG, vp, vn, bad, mat, bvh, "material")
    m = mat.copy(); m[6] = 7.0                                           # material type the kernel lacks
    _expect(RT_ERR_SCENE, vp, vn, face, m, bvh, "type")
    m = mat.copy(); m[0] = np.nan
    _expect(RT_ERR_SCENE, vp, vn, face, m, bvh, "type")


@pytest.mark.parametrize("mutate,match", [
    (lambda b: b.__setitem__(0, 0.0), "cycle"),                # root's left child is the root
    (lambda b: b.__setitem__(9 * 1 + 1, 0.0), "cycle"),        # node 1's right child is the root
    (lambda b: b.__setitem__(0, 1e9), "out of range"),
    (lambda b: b.__setitem__(1, np.nan), "out of range"),
    (lambda b: b.__setitem__(8, 36.0), "out of range"),        # triangle index = triangle count
    (lambda b: b.__setitem__(1, -7.0), "out of range"),
])
def test_scene_check_refuses_malformed_bvh(mutate, match):
    sc = _cornell()
    b = sc.BVH.exportArray.copy()
    mutate(b)
    _expect(RT_ERR_SCENE, sc.V_p, sc.V_n, sc.faceData, sc.materialData, b, match)


def test_scene_check_shapes_the_reference_kernel_walks_but_fast_cannot():
    # a node reachable twice (a DAG, no cycle): the reference walks it twice; the FAST layouts need a
    # tree, so the scene is accepted with the REF traversal only
    sc = _cornell()
    b = sc.BVH.exportArray.copy().reshape(-1, 9)
    l0, r0 = int(b[0, 0]), int(b[0, 1])
    b[r0, 0] = b[l0, 0]                  # the right subtree shares the left subtree's left child
    info = _native.scene_check(sc.V_p, sc.V_n, sc.faceData, sc.materialData, b.ravel())
    assert not info["fast_ok"] and "FAST traversal unavailable" in info["note"]


def test_scene_check_non_finite_geometry():
    # NaN / inf vertices and boxes: the arrays are index-valid, so they are accepted; the packer must
    # neither fault nor loop (the SAH binning and the 4-wide quantisation see non-finite bounds)
    sc = _cornell()
    vp = sc.V_p.copy(); vp[:6] = [np.nan, np.inf, -np.inf, np.nan, 0, 0]
    b = sc.BVH.exportArray.copy().reshape(-1, 9)
    b[1:, 2:8][::3] = np.nan
    b[2:, 2:8][::5] = np.inf
    info = _native.scene_check(vp, sc.V_n, sc.faceData, sc.materialData, b.ravel())
    assert info["tris"] == 36
    big = W.CONFIGS["C1"].inputs()[0]
    # a larger tree through the binned SAH path (> 64 leaves) with NaN leaf boxes
    g = W.grid_obj_text(12)
    vp, vn, vuv, face, _ = _native.parse_obj(g)
    exp = B.build_export_array(face, vp).reshape(-1, 9)
    leaves = np.nonzero(exp[:, 8] >= 0)[0]
    exp[leaves[::7], 2:8] = np.nan
    exp[leaves[1::11], 2:5] = -np.inf
    info = _native.scene_check(vp, vn, face, big.materialData[:6], exp.ravel())
    assert info["tris"] == face.size // 10
    info = _native.scene_check(vp, vn, face, big.materialData[:6], exp.ravel(), layout=_native.RT_BVH_REFERENCE)
    assert info["tris"] == face.size // 10


def test_scene_check_empty_scene():
    info = _native.scene_check(np.zeros(0, np.float32), np.zeros(0, np.float32), np.zeros(0, np.int32),
                               np.array([1, 1, 1, 1, 0, 0], np.float32), np.zeros(0, np.float32))
    assert info["tris"] == 0
