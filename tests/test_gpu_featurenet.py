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


@pytest.mark.parametrize("cout,bn,relu,h,w", [(32, True, True, 20, 28), (16, False, False, 37, 45),
                                              (8, True, False, 9, 70), (32, False, True, 64, 48)])
def test_dcn_fused_vs_oracle(cout, bn, relu, h, w):
    """tmvs_dcn_fused: conv_offset_mask (3x3, 32 -> 27, bias) in-kernel + deform_conv2d, against the
    oracle's F.conv2d + deform_conv2d. Offsets of several pixels (samples beyond the LDS window take
    the global fallback), ragged H/W (partial 16-pixel steps and 8-row bands). Tolerance: the DCN's
    2e-5 abs + 1e-5 rel, widened to 5e-5 abs since the offsets themselves carry MFMA-order rounding."""
    torch.manual_seed(100 + cout + h)
    b = 2
    x = torch.randn(b, 32, h, w)
    wom = torch.randn(27, 32, 3, 3) * 0.05
    bom = torch.randn(27) * 0.5
    weight = torch.randn(cout, 32, 3, 3) * 0.06
    bias = torch.randn(cout) * 0.1
    om = F.conv2d(x, wom, bom, padding=1)
    ref = oracle.deform_conv2d(x, om[:, :18], weight, bias, 1, torch.sigmoid(om[:, 18:]))
    fold = None
    if bn:
        gamma, beta = torch.rand(cout) + 0.5, torch.randn(cout) * 0.1
        mean, var = torch.randn(cout) * 0.1, torch.rand(cout) + 0.5
        ref = F.batch_norm(ref, mean, var, gamma, beta, False, 0.1, 1e-5)
        a, s_ = ops.bn_fold(gamma, beta, mean, var)
        fold = (torch.from_numpy(a).to(DEV), torch.from_numpy(s_).to(DEV))
    if relu:
        ref = F.relu(ref)
    out, out_nhwc = ops.dcn_fused(x.permute(0, 2, 3, 1).contiguous().to(DEV), ops.deform_conv2d_pack(wom).to(DEV),
                                  bom.to(DEV), ops.deform_conv2d_pack(weight).to(DEV), bias.to(DEV), cout, bn=fold,
                                  relu=relu, want_nchw=True, want_nhwc=True)
    np.testing.assert_allclose(to_np(out), to_np(ref), rtol=1e-5, atol=5e-5)
    np.testing.assert_array_equal(to_np(out_nhwc), to_np(out.permute(0, 2, 3, 1)))


def test_dcn_fused_zero_offsets_is_masked_conv():
    """The reference's initial state (zero offset/mask conv, models/dcn.py:62-64): every tap samples an
    integer position with mask sigmoid(0) = 0.5, i.e. 0.5 * conv2d(x, W) + bias."""
    torch.manual_seed(7)
    x = torch.randn(3, 32, 24, 40)
    weight = torch.randn(32, 32, 3, 3) * 0.06
    bias = torch.randn(32) * 0.1
    ref = F.conv2d(0.5 * x, weight, bias, padding=1)
    out, _ = ops.dcn_fused(x.permute(0, 2, 3, 1).contiguous().to(DEV),
                           ops.deform_conv2d_pack(torch.zeros(27, 32, 3, 3)).to(DEV), torch.zeros(27, device=DEV),
                           ops.deform_conv2d_pack(weight).to(DEV), bias.to(DEV), 32)
    np.testing.assert_allclose(to_np(out), to_np(ref), rtol=1e-5, atol=2e-5)


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


def test_conv3x3_nhwc_bn_relu():
    """tmvs_conv3x3_nhwc = Conv2d(32, 32, 3, 1, 1, bias=False) -> eval BN -> ReLU (models/module.py:24-61),
    ragged sizes; 2e-5 abs + 1e-5 rel (MFMA K-order vs the CPU conv)."""
    torch.manual_seed(3)
    for (b, h, w) in ((2, 20, 28), (1, 9, 70), (3, 33, 17)):
        x = torch.randn(b, 32, h, w)
        weight = torch.randn(32, 32, 3, 3) * 0.06
        gamma, beta = torch.rand(32) + 0.5, torch.randn(32) * 0.1
        mean, var = torch.randn(32) * 0.1, torch.rand(32) + 0.5
        ref = F.relu(F.batch_norm(F.conv2d(x, weight, padding=1), mean, var, gamma, beta, False, 0.1, 1e-5))
        a, s_ = ops.bn_fold(gamma, beta, mean, var)
        fold = (torch.from_numpy(a).to(DEV), torch.from_numpy(s_).to(DEV))
        out, out_nhwc = ops.conv3x3_nhwc(x.permute(0, 2, 3, 1).contiguous().to(DEV), ops.deform_conv2d_pack(weight).to(DEV),
                                         bn=fold, relu=True, want_nchw=True, want_nhwc=True)
        np.testing.assert_allclose(to_np(out), to_np(ref), rtol=1e-5, atol=2e-5)
        np.testing.assert_array_equal(to_np(out_nhwc), to_np(out.permute(0, 2, 3, 1)))


@pytest.mark.parametrize("cl", [8, 16])
def test_fpn_merge(cl):
    """tmvs_fpn_merge = interpolate(prev, 2, nearest) + Conv2d(cl, 32, 1, bias) (models/module.py:413,417)."""
    torch.manual_seed(cl)
    b, h, w = 2, 11, 13
    prev = torch.randn(b, 32, h, w)
    lat = torch.randn(b, cl, 2 * h, 2 * w)
    conv = torch.nn.Conv2d(cl, 32, 1, bias=True)
    with torch.no_grad():
        ref = F.interpolate(prev, scale_factor=2.0, mode="nearest") + conv(lat)
    out = ops.fpn_merge(prev.permute(0, 2, 3, 1).contiguous().to(DEV), lat.permute(0, 2, 3, 1).contiguous().to(DEV),
                        conv.weight.detach().reshape(32, cl).contiguous().to(DEV), conv.bias.detach().to(DEV))
    np.testing.assert_allclose(to_np(out), to_np(ref.permute(0, 2, 3, 1)), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("cin,cout,k,stride,h,w", [(3, 8, 3, 1, 37, 50), (8, 8, 3, 1, 20, 33), (8, 16, 5, 2, 41, 70),
                                                   (16, 16, 3, 1, 17, 40), (16, 32, 5, 2, 36, 48),
                                                   (32, 32, 3, 1, 19, 21), (32, 32, 1, 1, 9, 35)])
def test_conv2d_bn_relu_shapes(cin, cout, k, stride, h, w):
    """tmvs_conv2d_bn_relu for every FeatureNet Conv2d block shape (models/module.py:349-362): Conv2d(k,
    stride, padding k//2, no bias) -> eval BN -> ReLU, ragged sizes; the first layer reads the NCHW
    image. 2e-5 abs + 1e-5 rel (MFMA K-order vs the CPU conv)."""
    torch.manual_seed(cin * 7 + cout + k)
    b = 2
    x = torch.randn(b, cin, h, w)
    weight = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
    gamma, beta = torch.rand(cout) + 0.5, torch.randn(cout) * 0.1
    mean, var = torch.randn(cout) * 0.1, torch.rand(cout) + 0.5
    ref = F.relu(F.batch_norm(F.conv2d(x, weight, stride=stride, padding=k // 2), mean, var, gamma, beta, False, 0.1,
                              1e-5))
    a, s_ = ops.bn_fold(gamma, beta, mean, var)
    fold = (torch.from_numpy(a).to(DEV), torch.from_numpy(s_).to(DEV))
    xin = x.contiguous() if cin == 3 else x.permute(0, 2, 3, 1).contiguous()
    out = ops.conv2d_bn_relu(xin.to(DEV), ops.conv2d_pack(weight).to(DEV), cout, k, stride, bn=fold, relu=True,
                             nchw_input=(cin == 3))
    np.testing.assert_allclose(to_np(out), to_np(ref.permute(0, 2, 3, 1)), rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("cout,h,w,scale", [(32, 20, 28, 2.5), (16, 37, 45, 1.0), (8, 9, 70, 4.0), (32, 33, 40, 0.3)])
def test_dcn_backward_vs_autograd(cout, h, w, scale):
    """tmvs_dcn_backward (dx scatter, d offsets / mask logits, dW) against fp64 autograd through the
    oracle's deform_conv2d. Offsets of `scale` std: at 2.5 / 4.0 many corners fall beyond the LDS
    window's R = 2 px halo (the global-atomic path) and outside the image; one corner region sits at
    exact integer positions (right-sided bilinear derivative, as torchvision's backward).
    Bar: 2e-5 of each gradient's max |value| (fp32 dot products of <= 288 terms vs exact)."""
    from transmvsnet_amd.featurenet_train import _taps, _untaps
    torch.manual_seed(cout + h)
    b = 2
    x = torch.randn(b, 32, h, w, dtype=torch.float64)
    om = torch.randn(b, 27, h, w, dtype=torch.float64)
    om[:, :18] *= scale
    om[0, :18, :3, :3] = 0.0
    weight = torch.randn(cout, 32, 3, 3, dtype=torch.float64) * 0.06
    dy = torch.randn(b, cout, h, w, dtype=torch.float64)
    x32, om32, w32 = x.float(), om.float(), weight.float()
    # the exact reference: fp64 autograd at the fp32-rounded inputs
    xr = x32.double().requires_grad_(True)
    offr = om32[:, :18].double().requires_grad_(True)
    mlr = om32[:, 18:].double().requires_grad_(True)
    wr = w32.double().requires_grad_(True)
    out = oracle.deform_conv2d(xr, offr, wr, None, 1, torch.sigmoid(mlr))
    (out * dy.float().double()).sum().backward()
    dx = torch.zeros(b, h, w, 32, device=DEV)
    dom, dw = ops.dcn_backward(x32.permute(0, 2, 3, 1).contiguous().to(DEV), om32.contiguous().to(DEV),
                               _taps(w32).to(DEV), dy.float().permute(0, 2, 3, 1).contiguous().to(DEV), dx)
    torch.cuda.synchronize()

    def close(got, ref, tag):
        ref = ref.detach()
        err = float((got.double().cpu() - ref).abs().max()) / max(float(ref.abs().max()), 1e-30)
        assert err <= 2e-5, (tag, err)

    close(dx.permute(0, 3, 1, 2), xr.grad, "dx")
    close(dom[..., :18].permute(0, 3, 1, 2), offr.grad, "d offset")
    close(dom[..., 18:27].permute(0, 3, 1, 2), mlr.grad, "d mask logit")
    assert float(dom[..., 27:].abs().max()) == 0.0
    close(_untaps(dw, tuple(weight.shape)), wr.grad, "dW")
    # determinism: the in-window scatter is integer (order-free); a second call gives the same bits
    # when no corner leaves the window
    if scale <= 0.3:
        dx2 = torch.zeros_like(dx)
        ops.dcn_backward(x32.permute(0, 2, 3, 1).contiguous().to(DEV), om32.contiguous().to(DEV),
                         _taps(w32).to(DEV), dy.float().permute(0, 2, 3, 1).contiguous().to(DEV), dx2)
        assert torch.equal(dx, dx2)


@pytest.mark.parametrize("a,bc,k,stride,h,w", [(32, 32, 3, 1, 37, 70), (27, 32, 3, 1, 20, 33), (16, 16, 3, 1, 9, 40),
                                               (16, 8, 3, 2, 24, 30), (32, 16, 1, 1, 13, 17), (16, 32, 1, 1, 36, 48),
                                               (8, 16, 1, 1, 72, 96), (8, 8, 3, 1, 144, 192)])
def test_conv2d_wgrad_vs_torch(a, bc, k, stride, h, w):
    """tmvs_conv2d_wgrad (dW[k][a][b] = sum_p dz[p][a] x[p*s - pad + k][b]) against torch's fp64 conv2d
    weight gradient, incl. the all-taps 3x3 kernel (32 x 32, ragged tiles) and the 27-row offset conv.
    Bar: 1e-5 of max |dW| (fp32 products summed over <= 10^4 pixels per tile, fp64 across tiles)."""
    from torch.nn.grad import conv2d_weight
    torch.manual_seed(a + bc + k + h)
    pad = k // 2
    b = 3
    x = torch.randn(b, bc, h, w, dtype=torch.float64)
    ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    dz = torch.randn(b, a, ho, wo, dtype=torch.float64)
    ref = conv2d_weight(x, (a, bc, k, k), dz, stride=stride, padding=pad)  # [a][bc][k][k]
    dw = ops.conv2d_wgrad(dz.float().permute(0, 2, 3, 1).contiguous().to(DEV),
                          x.float().permute(0, 2, 3, 1).contiguous().to(DEV), k, stride, pad)  # [k*k][a][bc]
    got = dw.double().cpu().reshape(k, k, a, bc).permute(2, 3, 0, 1)
    err = float((got - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err


@pytest.mark.parametrize("scale", [0.3, 4.0])
def test_dcn_backward_set_matches_accumulate_form(scale):
    """tmvs_dcn_backward_set (dx written; the corners beyond the windows through the self-clearing far buffer)
    against tmvs_dcn_backward into a zeroed dx: bitwise when no corner leaves the window (0.3 px), within fp32
    atomic-order rounding otherwise (4 px), and the far buffer is all zero again after each call (twice)."""
    from transmvsnet_amd.featurenet_train import _taps
    torch.manual_seed(11)
    b, h, w, cout = 2, 30, 44, 32
    x = torch.randn(b, h, w, 32, device=DEV)
    om = torch.randn(b, 27, h, w, device=DEV)
    om[:, :18] *= scale
    wt = _taps(torch.randn(cout, 32, 3, 3) * 0.06).to(DEV)
    dy = torch.randn(b, h, w, cout, device=DEV)
    dx_ref = torch.zeros(b, h, w, 32, device=DEV)
    dom_ref, dw_ref = ops.dcn_backward(x, om.contiguous(), wt, dy, dx_ref)
    for _ in range(2):
        dx, dom, dw = ops.dcn_backward_set(x, om.contiguous(), wt, dy)
        torch.cuda.synchronize()
        far = ops._DCN_FAR[(str(x.device), tuple(x.shape))][0]
        assert float(far.abs().max()) == 0.0
        assert torch.equal(dom, dom_ref) and torch.equal(dw, dw_ref)
        if scale <= 0.3:
            assert torch.equal(dx, dx_ref)
        else:
            err = float((dx - dx_ref).abs().max()) / float(dx_ref.abs().max())
            assert err <= 1e-6, err


def test_dcn_backward_set_first_call_inside_capture_raises():
    """The far buffer of a new shape is allocated and zeroed outside any HIP-graph capture: a first call for a
    shape inside a capture raises (a fill recorded in the graph would run per replay, and an eager call before
    the first replay would read an unfilled buffer); after one eager call the same shape captures."""
    from transmvsnet_amd.featurenet_train import _taps
    torch.manual_seed(12)
    b, h, w, cout = 1, 14, 22, 8
    x = torch.randn(b, h, w, 32, device=DEV)
    om = torch.randn(b, 27, h, w, device=DEV).contiguous()
    wt = _taps(torch.randn(cout, 32, 3, 3) * 0.06).to(DEV)
    dy = torch.randn(b, h, w, cout, device=DEV)
    assert (str(x.device), tuple(x.shape)) not in ops._DCN_FAR
    g = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match="outside any capture"):
        with torch.cuda.graph(g):
            ops.dcn_backward_set(x, om, wt, dy)
    dx0, _, _ = ops.dcn_backward_set(x, om, wt, dy)  # eager: creates the buffer
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        dx1, _, _ = ops.dcn_backward_set(x, om, wt, dy)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)


def test_dcn_backward_nonfinite_dy_poisons_dx():
    """A non-finite upstream gradient (inf / NaN in dy) makes tmvs_dcn_backward's dx and d offset/mask
    non-finite (the kFixBad path: the fixed-point window cannot hold it, so every window is written
    as NaN), so the training step's overflow / finiteness checks see it."""
    from transmvsnet_amd.featurenet_train import _taps
    torch.manual_seed(3)
    b, h, w, cout = 1, 24, 40, 32
    x = torch.randn(b, h, w, 32, device=DEV)
    om = torch.randn(b, 27, h, w, device=DEV) * 0.3
    wt = _taps(torch.randn(cout, 32, 3, 3) * 0.06).to(DEV)
    for bad in (float("inf"), float("nan")):
        dy = torch.randn(b, h, w, cout, device=DEV)
        dy[0, 5, 7, 3] = bad
        dx = torch.zeros(b, h, w, 32, device=DEV)
        dom, dw = ops.dcn_backward(x, om.contiguous(), wt, dy, dx)
        torch.cuda.synchronize()
        assert not bool(torch.isfinite(dx).all()), bad
        assert not bool(torch.isfinite(dom[..., :27]).all()), bad
