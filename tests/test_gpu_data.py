"""Input side on the GPU: scans in the reference's on-disk layout, loaded by
transmvsnet_amd.data (DTU: load_sample = general_eval.py:126-210; Tanks&Temples: load_sample_tnt =
tnt_eval.py:120-210), fed to TransMVSNet.forward (HIP, FeatureNet included) and compared with the
oracle's forward on the same loaded arrays. Depth parity: flips only at reference near-ties (top-2
log-prob margin < 1e-4) and mean |Δdepth| <= 1e-4 mm. The cv2 resize restatement is not exercised
here (the images already have the target size): it stays parity-unpinned (cv2 absent).
"""
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle import transmvs_ref as oracle
from tests._util import depth_parity, golden_state_dict, to_np
from tests.test_data_io import _write_scan
from transmvsnet_amd import TransMVSNet, data

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def sd():
    return golden_state_dict()


def _forward_parity(sd, sample, ndepths):
    m = TransMVSNet(ndepths=list(ndepths)).eval()
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    imgs = torch.from_numpy(sample["imgs"])[None]
    proj = {k: torch.from_numpy(v)[None] for k, v in sample["proj_matrix"].items()}
    dv = torch.from_numpy(sample["depth_values"])[None]
    with torch.no_grad():
        out = m(imgs.to(DEV), proj, dv.to(DEV))
        ref = oracle.forward(sd, imgs, proj, dv, ndepths=tuple(ndepths))
    for s in (1, 2, 3):
        mean_l1, near, flips = depth_parity(to_np(out[f"stage{s}"]["depth"]), to_np(ref[f"stage{s}"]["depth"]),
                                            to_np(ref[f"stage{s}"]["prob_volume"]))
        assert flips == 0, (s, mean_l1, near, flips)
    l1 = float(np.abs(to_np(out["depth"]).astype(np.float64) - to_np(ref["depth"]).astype(np.float64)).mean())
    assert l1 <= 1e-4, l1
    return l1


def test_dtu_scan_loaded_and_forwarded(sd):
    with tempfile.TemporaryDirectory() as td:
        _write_scan(td, "scan1", 5, "cams", h=300, w=400, seed=4)
        metas = data.read_pair_file(os.path.join(td, "scan1", "pair.txt"), nviews=4)
        ref_view, src = metas[0]
        sample = data.load_sample(td, "scan1", ref_view, src, nviews=5)
    assert sample["imgs"].shape == (5, 3, 288, 384)
    print("DTU-layout scan -> forward: depth L1 vs oracle", _forward_parity(sd, sample, (48, 32, 8)))


def test_tnt_scan_loaded_and_forwarded(sd):
    with tempfile.TemporaryDirectory() as td:
        _write_scan(td, "Horse", 3, "cams_1", h=300, w=400, tnt=True, seed=5)
        metas = data.read_pair_file(os.path.join(td, "Horse", "pair.txt"), pad=False)
        ref_view, src = metas[1]
        sample = data.load_sample_tnt(td, "Horse", ref_view, src, nviews=11)
    assert sample["imgs"].shape == (3, 3, 288, 384)  # nviews shrinks to 1 + 2 sources
    print("TnT-layout scan -> forward: depth L1 vs oracle", _forward_parity(sd, sample, (48, 32, 8)))
