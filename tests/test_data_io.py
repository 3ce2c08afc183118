"""Input side: the reference's dataset readers (transmvsnet_amd/data.py).

PFM: pinned byte-for-byte to files written by the reference's own datasets/data_io.py
(tests/golden/pfm.npz, tests/golden/make_golden_io.py). Scan files: the reference ships none, so
the DTU / TnT cam and pair formats are exercised through files written here in the documented
layout (general_eval.py:69-80, 41-56) and checked against the reference's arithmetic. The resize
(cv2.resize INTER_LINEAR; cv2 absent) is parity-unpinned: checked against torch's bilinear
interpolation with the same half-pixel convention (1e-5; torch orders its lerp differently).
"""
import os
import tempfile

import numpy as np
import torch
import torch.nn.functional as F

from tests._util import golden
from transmvsnet_amd import data

CAM_TXT = """extrinsic
0.970263 0.00747983 0.241939 -191.02
-0.0147429 0.999493 0.0282234 3.28832
-0.241605 -0.030951 0.969881 22.5401
0.0 0.0 0.0 1.0

intrinsic
2892.33 0 823.205
0 2883.18 619.071
0 0 1

425.0 2.5
"""

PAIR_TXT = """3
0
10 10 2346.41 1 2036.53 9 1243.89 12 1052.87 11 1000.84 13 703.583 2 604.456 8 439.759 14 327.419 27 249.278
1
2 5 10.0 6 9.0
2
0
"""


def test_pfm_matches_reference_bytes():
    g = golden("pfm.npz")
    with tempfile.TemporaryDirectory() as td:
        for name in ("grey", "colour"):
            fn = os.path.join(td, name + ".pfm")
            data.save_pfm(fn, g[name + "_in"].copy())
            assert open(fn, "rb").read() == g[name + "_bytes"].tobytes(), name
            ref_fn = os.path.join(td, name + "_ref.pfm")
            g[name + "_bytes"].tofile(ref_fn)
            back, scale = data.read_pfm(ref_fn)
            np.testing.assert_array_equal(back, g[name + "_read"])
            assert scale == float(g[name + "_scale"])


def test_read_pair_file_fills_sources():
    with tempfile.TemporaryDirectory() as td:
        fn = os.path.join(td, "pair.txt")
        open(fn, "w").write(PAIR_TXT)
        metas = data.read_pair_file(fn, nviews=5)
    assert metas == [(0, [10, 1, 9, 12, 11, 13, 2, 8, 14, 27]), (1, [5, 6, 5, 5, 5])]  # view 2: no sources


def test_read_cam_file_dtu_and_tnt():
    with tempfile.TemporaryDirectory() as td:
        fn = os.path.join(td, "00000000_cam.txt")
        open(fn, "w").write(CAM_TXT)
        k, e, dmin, dint = data.read_cam_file(fn)
        np.testing.assert_allclose(k[0], np.float32([2892.33, 0, 823.205]) / 4)
        assert k.dtype == np.float32 and k[2, 2] == 1.0 and e[0, 3] == np.float32(-191.02)
        assert (dmin, dint) == (425.0, 2.5)
        open(fn, "w").write(CAM_TXT.replace("425.0 2.5", "425.0 2.5 192"))
        assert data.read_cam_file(fn, ndepths=96)[3] == (425.0 + 192 * 2.5 - 425.0) / 96
        open(fn, "w").write(CAM_TXT.replace("425.0 2.5", "1.5 9.5"))
        *_, dmin, dint, dmax = data.read_cam_file(fn, ndepths=192, tnt=True)
        assert (dmin, dmax) == (1.5, 9.5) and dint == 8.0 / 192


def test_scale_mvs_input_dtu():
    img = np.random.default_rng(0).random((1200, 1600, 3)).astype(np.float32)
    k = np.array([[723.08, 0, 205.8], [0, 720.8, 154.77], [0, 0, 1]], np.float32)
    out, k2 = data.scale_mvs_input(img, k, 1152, 864)
    assert out.shape == (864, 1152, 3)
    np.testing.assert_allclose(k2[0], k[0] * 0.72, rtol=1e-6)
    np.testing.assert_allclose(k2[1], k[1] * 0.72, rtol=1e-6)


def test_resize_bilinear_half_pixel():
    img = np.random.default_rng(1).random((50, 70, 3)).astype(np.float32)
    for (nw, nh) in ((35, 25), (96, 64), (70, 50)):
        got = data.resize_bilinear(img, nw, nh)
        ref = F.interpolate(torch.from_numpy(img).permute(2, 0, 1)[None], size=(nh, nw), mode="bilinear",
                            align_corners=False)[0].permute(1, 2, 0).numpy()
        np.testing.assert_allclose(got, ref, atol=1e-5)  # same sample points; fp32 lerp order differs


def test_load_sample_synthetic_scan():
    from PIL import Image
    rng = np.random.default_rng(2)
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, "scan1", "images"))
        os.makedirs(os.path.join(td, "scan1", "cams"))
        for v in range(4):
            Image.fromarray((rng.random((300, 400, 3)) * 255).astype(np.uint8)).save(
                os.path.join(td, "scan1", "images", "{:0>8}.jpg".format(v)))
            open(os.path.join(td, "scan1", "cams", "{:0>8}_cam.txt".format(v)), "w").write(CAM_TXT)
        s = data.load_sample(td, "scan1", 0, [1, 2, 3], nviews=4, max_h=216, max_w=288)
    assert s["imgs"].shape == (4, 3, 192, 288)  # 300x400 -> x0.72 -> 216x288 -> multiples of 32: 192x288
    p1, p3 = s["proj_matrix"]["stage1"], s["proj_matrix"]["stage3"]
    np.testing.assert_allclose(p3[:, 1, :2, :], p1[:, 1, :2, :] * 4)
    np.testing.assert_allclose(p1[0, 1, 0, 0], 2892.33 / 4 * 288 / 400, rtol=1e-6)
    np.testing.assert_allclose(p1[0, 1, 1, 1], 2883.18 / 4 * 192 / 300, rtol=1e-6)
    assert len(s["depth_values"]) == 192 and s["depth_values"][1] == np.float32(427.5)


def _write_scan(td, scan, n_views, cams_dir, h=300, w=400, tnt=False, seed=3):
    """A scan directory in the reference's layout: images/{:08}.jpg, <cams_dir>/{:08}_cam.txt
    (per-view translated camera), pair.txt."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(td, scan, "images"), exist_ok=True)
    os.makedirs(os.path.join(td, scan, cams_dir), exist_ok=True)
    for v in range(n_views):
        Image.fromarray((rng.random((h, w, 3)) * 255).astype(np.uint8)).save(
            os.path.join(td, scan, "images", "{:0>8}.jpg".format(v)))
        lines = CAM_TXT.splitlines()
        row = lines[1].split()
        row[3] = "%.3f" % (float(row[3]) + 40.0 * v)
        lines[1] = " ".join(row)
        if tnt:
            lines[11] = "425.0 935.0"
        open(os.path.join(td, scan, cams_dir, "{:0>8}_cam.txt".format(v)), "w").write("\n".join(lines) + "\n")
    with open(os.path.join(td, scan, "pair.txt"), "w") as f:
        f.write(f"{n_views}\n")
        for v in range(n_views):
            src = [u for u in range(n_views) if u != v]
            f.write(f"{v}\n{len(src)} " + " ".join(f"{u} {10.0 - u:.1f}" for u in src) + "\n")


def test_read_pair_file_tnt_no_padding():
    with tempfile.TemporaryDirectory() as td:
        fn = os.path.join(td, "pair.txt")
        open(fn, "w").write(PAIR_TXT)
        metas = data.read_pair_file(fn, nviews=11, pad=False)
    assert metas == [(0, [10, 1, 9, 12, 11, 13, 2, 8, 14, 27]), (1, [5, 6])]  # view 2 has no sources


def test_load_sample_tnt_shrinks_views_and_ranges():
    with tempfile.TemporaryDirectory() as td:
        _write_scan(td, "Family", 4, "cams_1", tnt=True)
        metas = data.read_pair_file(os.path.join(td, "Family", "pair.txt"), pad=False)
        s = data.load_sample_tnt(td, "Family", metas[0][0], metas[0][1], nviews=11)
        # an explicit cap for a scan outside the table, and the dataset-wide resolution carried over
        s2 = data.load_sample_tnt(td, "Family", 1, [0, 2], image_size=(256, 192), fixed_hw=s["fixed_hw"])
    assert s["imgs"].shape == (4, 3, 288, 384)  # 1 + 3 sources; 300x400 under 1920x1080 -> multiples of 32
    assert s2["imgs"].shape == (3, 3, 288, 384)  # resized back to the fixed resolution
    dint = (935.0 - 425.0) / 192
    np.testing.assert_array_equal(s["depth_values"], np.arange(425.0, dint * 192 + 425.0, dint, dtype=np.float32))
    p = s2["proj_matrix"]["stage1"]
    # 400x300 -> capped at 256x192 (x0.64: 256x192) -> back to 384x288: intrinsics x0.64 x1.5 x(1/4)
    np.testing.assert_allclose(p[0, 1, 0, 0], 2892.33 / 4 * (256 / 400) * (384 / 256), rtol=1e-6)
