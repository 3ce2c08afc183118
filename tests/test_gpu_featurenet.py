"""FeatureNet / DCNv2 HIP kernel vs the oracle (needs an MI355X; -m gpu).

The oracle restates torchvision.ops.deform_conv2d (torchvision 0.10.1; absent here). At the
reference's zero-initialised offsets it is exact (pinned by the e2e image goldens); for nonzero
offsets it follows torchvision's documented layout -- parity there is unpinned by the reference.
Tolerances: DCN outputs 2e-5 abs + 1e-5 rel (fp32 MFMA K-order vs the oracle's matmul);
FeatureNet stage features 1e-4 abs (several conv layers: MIOpen vs CPU conv order).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import transmvs_ref as oracle
from transmvsnet_amd import TransMVSNet, ops, synthetic
from tests._util import to_np

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("cout,bn,relu", [(32, True, True), (16, False, False), (8, False, False), (32, False, True)])
def test_deform_conv2d_random_offsets(cout, bn, relu):
    torch.manual_seed(cout + 2 * bn + relu)
    b, h, w = 2, 20, 28
    x = torch.randn(b, 32, h, w)
    om = torch.randn(b, 27, h, w)
    om[:, :18] *= 2.5  # offsets of a few pixels: samples straddle and leave the image
    om[0, :18, :3, :3] = 0.0  # and some exact integer positions
    weight = torch.randn(cout, 32, 3, 3) * 0.06
    bias = torch.randn(cout) * 0.1
    ref = oracle.deform_conv2d(x, om[:, :18], weight, bias, 1, torch.sigmoid(om[:, 18:]))
    fold = None
    if bn:
        gamma, beta = torch.rand(cout) + 0.5, torch.randn(cout) * 0.1
        mean, var = torch.randn(cout) * 0.1, torch.rand(cout) + 0.5
        ref = F.batch_norm(ref, mean, var, gamma, beta, False, 0.1, 1e-5)
        a, s = ops.bn_fold(gamma, beta, mean, var)
        fold = (torch.from_numpy(a).to(DEV), torch.from_numpy(s).to(DEV))
    if relu:
        ref = F.relu(ref)
    out, out_nhwc = ops.deform_conv2d(x.permute(0, 2, 3, 1).contiguous().to(DEV), om.contiguous().to(DEV),
                                      ops.deform_conv2d_pack(weight).to(DEV), bias.to(DEV), cout, bn=fold, relu=relu,
                                      want_nhwc=True)
    np.testing.assert_allclose(to_np(out), to_np(ref), rtol=1e-5, atol=2e-5)
    np.testing.assert_array_equal(to_np(out_nhwc), to_np(out.permute(0, 2, 3, 1)))


def test_featurenet_nonzero_offsets_vs_oracle():
    """Whole FeatureNet (3 scales, 9 DCNs) with trained-like nonzero offset/mask convs, 2 views batched."""
    m = TransMVSNet().eval()
    sd = synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=3, sharpen=1.0)
    g = torch.Generator().manual_seed(11)
    for k in sd:
        if "conv_offset_mask" in k:
            sd[k] = torch.randn(sd[k].shape, generator=g) * (0.05 if k.endswith("weight") else 0.5)
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    imgs = synthetic.synthetic_images(2, 64, 96, seed=5)[0]
    with torch.no_grad():
        out = m.feature(imgs.to(DEV))
        for v in range(2):
            ref = oracle.feature_net(sd, imgs[v:v + 1])
            for s in ("stage1", "stage2", "stage3"):
                np.testing.assert_allclose(to_np(out[s][v:v + 1]), to_np(ref[s]), rtol=0, atol=1e-4, err_msg=s)
