"""Depth-map fusion (gipuma/fusibile) and the output-side writers -- SURVEY.md 8f rank 4.

CPU tests: the host writers and camera decomposition against their reference formulas, the oracle
on a synthetic scene. GPU tests (-m gpu): tmvs_fusibile against the oracle (oracle/fusion_ref.py).
Parity unpinned by the reference (fusibile needs CUDA + OpenCV, absent; no fused clouds shipped).
Tolerances: float32 kernel vs float64 oracle. The kernel makes discrete decisions on rounded
values -- the 0.25 disparity threshold, floor() of the projected pixel (texel and 3D point), the
8-bit filter weights -- so a few pixels legitimately take the other branch: the fused mask may
differ on <= 0.2 % of pixels, and <= 2 % of the agreeing pixels may fall outside 1e-3 mm + 1e-5
rel (one view's neighbouring texel / pixel), all within 10 mm; colours likewise within 1e-5.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle import fusion_ref
from tests._fusion_scene import make_scene
from transmvsnet_amd import fusion


def test_depth_normal_and_decode():
    """utils.depth_normal (clamp to [425, 935], uint8 of (d - 425) / 510 * 255) and fusibile's
    425 + 512 * a / 255 decoding (main.cpp:136): the reference's 510-vs-512 scale mismatch is kept."""
    d = np.array([[100.0, 425.0, 600.0, 935.0, 2000.0]], np.float32)
    u = fusion.depth_normal(d)
    assert u.dtype == np.uint8
    np.testing.assert_array_equal(u, [[0, 0, 87, 255, 255]])
    dec = fusion.depth_decode(u)
    np.testing.assert_allclose(dec, [[425.0, 425.0, 425.0 + 512.0 * 87 / 255, 937.0, 937.0]], rtol=1e-6)


def test_write_read_cam_roundtrip():
    """test.write_cam writes P = K [R | t] (3 rows + blank line); fusibile reads 3 x 4 floats back."""
    _, _, _, ps = make_scene(v=2, h=16, w=24)
    with tempfile.TemporaryDirectory() as td:
        fn = os.path.join(td, "00000000.txt")
        k = np.zeros((4, 4), np.float32)
        k[:3, :3] = [[2080.0, 0, 576.0], [0, 2075.0, 432.0], [0, 0, 1]]
        e = np.eye(4, dtype=np.float32)
        e[:3, 3] = [-191.02, 3.28832, 22.5401]
        fusion.write_cam(fn, np.stack([e, k]))
        lines = open(fn).read().split("\n")
        assert len(lines) == 5 and lines[3] == "" and len(lines[0].split()) == 4
        np.testing.assert_allclose(fusion.read_cam(fn), (k @ e)[:3], rtol=1e-6)


def test_camera_params_recover_k_and_centre():
    """get_camera_parameters: fx from the RQ decomposition, C4 = the camera centre, RK_inv = inv(P33)."""
    rgbd, packs, dicts, ps = make_scene(v=3, h=16, w=24)
    for p, d, pk in zip(ps, dicts, packs):
        k, r = fusion._rq3(p[:, :3].astype(np.float64))
        np.testing.assert_allclose(k @ r, p[:, :3], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(r @ r.T, np.eye(3), atol=1e-9)
        assert abs(d["fx"] - 1.8 * 24) < 1e-3
        c_h = np.append(d["C4"], 1.0)
        np.testing.assert_allclose(p @ c_h, 0.0, atol=1e-2)  # P C = 0
        np.testing.assert_allclose(pk[:12], p.reshape(-1).astype(np.float32))
        np.testing.assert_allclose(d["RK_inv"] @ p[:, :3], np.eye(3), atol=1e-5)


def test_oracle_fuses_consistent_scene():
    """The restated fusibile on a scene whose views agree: most valid pixels fuse, the
    fused points lie on the plane n . X = 650, and the invalid-depth patch never fuses."""
    rgbd, packs, dicts, _ = make_scene()
    wr, cx, ct = fusion_ref.fusibile_ref(rgbd, dicts, 0)
    valid = rgbd[0, ..., 3] > fusion_ref.DEPTH_FLOOR
    assert wr[valid].mean() > 0.6 and not wr[~valid].any()  # image borders leave the other views
    n = np.array([0.05, -0.03, 1.0])
    np.testing.assert_allclose(cx[wr] @ n, 650.0, atol=5.0)  # 8-bit depth alpha: 2 mm steps
    assert np.all((ct[wr] >= 0) & (ct[wr] <= 1))


def test_save_point_cloud_format():
    """displayUtils.h save_point_cloud: binary little-endian PLY, 15 bytes per vertex, RGB from
    texture [2, 1, 0], non-finite coordinates written as 0."""
    x = np.array([[1.0, 2.0, 3.0], [np.inf, 1.0, 1.0]], np.float32)
    t = np.array([[0.1, 0.2, 0.3], [1.0, 0.0, 0.5]], np.float32)
    with tempfile.TemporaryDirectory() as td:
        fn = os.path.join(td, "3d_model.ply")
        fusion.save_point_cloud(fn, x, t)
        raw = open(fn, "rb").read()
    head, body = raw.split(b"end_header\n")
    assert b"element vertex 2" in head and len(body) == 2 * 15
    rec = np.frombuffer(body, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("r", "u1"), ("g", "u1"),
                                     ("b", "u1")])
    assert tuple(rec[0])[:3] == (1.0, 2.0, 3.0) and tuple(rec[0])[3:] == (76, 51, 25)
    assert tuple(rec[1])[:3] == (0.0, 0.0, 0.0) and tuple(rec[1])[3:] == (127, 0, 255)


def _close_mostly(got, want, atol, worst, rtol=1e-5, frac=0.02):
    err = np.abs(got.astype(np.float64) - want).max(axis=-1)
    bad = err > atol + rtol * np.abs(want).max(axis=-1)
    assert bad.mean() <= frac, (bad.mean(), err.max())
    assert err.max() <= worst, err.max()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(6, 96, 128), (4, 61, 83)])
def test_fusibile_kernel_vs_oracle(shape):
    """tmvs_fusibile for every reference camera against the oracle (fresh buffers)."""
    from transmvsnet_amd import _lib, ops
    v, h, w = shape
    rgbd, packs, dicts, _ = make_scene(v=v, h=h, w=w, seed=v + h)
    dev = "cuda"
    rg = torch.from_numpy(rgbd).to(dev)
    cams = torch.from_numpy(packs).to(dev)
    lib = _lib.load()
    for ref in range(v):
        coord = torch.zeros(h, w, 4, device=dev)
        tex = torch.zeros(h, w, 4, device=dev)
        _lib.check(lib.tmvs_fusibile(rg.data_ptr(), cams.data_ptr(), v, h, w, ref, 3, 0.25, coord.data_ptr(),
                                     tex.data_ptr(), ops._stream()), "tmvs_fusibile")
        coord, tex = coord.cpu().numpy(), tex.cpu().numpy()
        wr, cx, ct = fusion_ref.fusibile_ref(rgbd, dicts, ref)
        got = coord[..., 2] != 0
        assert (got != wr).mean() <= 2e-3, (ref, (got != wr).mean())
        both = got & wr
        assert both.sum() > 0.5 * wr.sum()
        _close_mostly(coord[both][:, :3], cx[both], 1e-3, 10.0)
        _close_mostly(tex[both][:, :3], ct[both], 1e-5, 0.5)
        assert np.all(coord[got][:, 3] == 0) and np.all(tex[got][:, 3] == 0)


@pytest.mark.gpu
def test_fuse_point_list_vs_oracle():
    """fusion.fuse (persistent buffer across cameras + pixel-order compaction, as the reference)
    against oracle.fuse_ref: same point count within 0.2 %, same point set where counts agree."""
    rgbd, packs, dicts, _ = make_scene(v=5, h=72, w=96, seed=3)
    xs, ts = fusion.fuse(torch.from_numpy(rgbd).cuda(), packs)
    rx, rt = fusion_ref.fuse_ref(rgbd, dicts)
    assert abs(len(xs) - len(rx)) <= 0.002 * len(rx) + 2
    if len(xs) == len(rx):
        _close_mostly(xs.cpu().numpy(), rx, 1e-3, 10.0)
        _close_mostly(ts.cpu().numpy(), rt, 1e-5, 0.5)
