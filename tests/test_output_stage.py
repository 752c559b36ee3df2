"""Output stage and IBL input, host side: the oracle's restatement of
FileManager.saveImg, the PNG writer and the IBL loader.  The device quantizer is covered by the
gpu tests (test_gpu_parity.py::test_rgb8_*)."""
import os

import numpy as np
import pytest

import oracle.oracle as O
from ensem3a_openclraytracer_amd import output
from ensem3a_openclraytracer_amd import workloads as W

REF = "/root/reference"


def test_oracle_rgb8_is_numpy_savimg_arithmetic():
    x = np.array([0.0, 1.0, 0.5, 1 / 255, np.nextafter(np.float32(1 / 255), np.float32(0)), 0.999999],
                 np.float32)
    got = O.rgb8(x)
    assert got.dtype == np.uint8
    # (x*255) in float32, truncated: 255*0.5 = 127.5 -> 127; 255*(1/255 rounded) -> 1 or 0 by rounding
    assert got.tolist()[:3] == [0, 255, 127]
    np.testing.assert_array_equal(got, (x * np.float32(255)).astype(np.uint8))


def test_save_img_writes_the_quantized_frame(tmp_path):
    rng = np.random.default_rng(3)
    frame = rng.random((16, 16, 3), dtype=np.float32)
    q = O.rgb8(frame)
    out = output.saveImg(q, 16, 16, str(tmp_path / "out"))       # uint8 input: no device needed
    from PIL import Image
    with Image.open(tmp_path / "out.png") as im:
        back = np.asarray(im.convert("RGB"))
    np.testing.assert_array_equal(back, q)
    np.testing.assert_array_equal(out, q)


def test_scene_ibl_resolves_the_iblfile_key(tmp_path):
    from PIL import Image
    img = np.zeros((4, 8, 3), np.uint8)
    img[1, 2] = (10, 20, 30)
    os.makedirs(tmp_path / "IBL")
    Image.fromarray(img, "RGB").save(tmp_path / "IBL" / "env.png")
    rgba = output.scene_ibl({"IBLfile": "IBL/env.png"}, str(tmp_path))
    assert rgba.shape == (4, 8, 4) and rgba.dtype == np.uint8
    assert rgba[1, 2].tolist() == [10, 20, 30, 255]
    with pytest.raises(FileNotFoundError, match="IBLfile"):
        output.scene_ibl({"IBLfile": "IBL/missing.jpg"}, str(tmp_path))


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_load_ibl_matches_the_bundled_preview_fixture():
    rgba = output.load_ibl(os.path.join(REF, "IBL", "Arches_E_PineTree_Preview.jpg"))
    np.testing.assert_array_equal(rgba, W.ibl_preview())
