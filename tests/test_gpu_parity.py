"""HIP path vs the CPU oracle / golden vectors (needs an MI355X; run with -m gpu).

Tolerances (fp32 throughout; stated per check, each with the deviation measured on the MI355X in
profiles/r05n/pytest_parity.log):
  * homo_warping seam: bit-exact (same op order, the fixtures' host rounding pinned)
  * cost volume similarity, PixelwiseNet view weights: 5e-7 abs (measured <= 1.5e-7: the channel-
    sum order of the correlation mean is the only difference, a few ulps)
  * pathway features: 3e-6 (measured 9.5e-7); FMT EncoderLayer tokens: 2e-6 (measured 7.2e-7;
    LayerNorm'd, O(1) values)
  * CostRegNet logits: 2e-5 relative to the volume's max |logit| (MFMA k-order vs mkldnn order)
  * probabilities: 1e-5 abs for a softmax of given logits; 2e-4 end to end (measured 8.4e-5: the
    sharpened logits, up to ~700, carry the CostRegNet deviation into the softmax)
  * hypotheses of the stage glue: bit-exact (same fp32 op sequence)
  * depth: identical argmax except at near-ties (top-2 log-prob margin < 1e-4),
    and mean |Δdepth| <= 1e-4 mm (the north-star bar)
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import transmvs_ref as oracle
from transmvsnet_amd import TransMVSNet, _lib, ops, synthetic
from tests._util import GOLDEN_ROT_ORDER, depth_parity, golden, golden_rot, golden_state_dict, to_np

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def sd():
    return golden_state_dict()


@pytest.fixture(scope="module")
def model(sd):
    m = TransMVSNet(ndepths=[8, 8, 8]).eval()
    m.load_state_dict(sd, strict=True)
    return m.to(DEV)


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _close(got, ref, atol, what):
    """assert max |got - ref| <= atol, printing the measured deviation (GPU logs keep the numbers)."""
    err = float(np.abs(np.asarray(got, np.float64) - np.asarray(ref, np.float64)).max())
    print(f"{what}: max abs err {err:.2e} (bound {atol:.0e})")
    assert err <= atol, (what, err, atol)


def test_library_loads_on_gpu():
    from transmvsnet_amd import _lib
    assert _lib.load().tmvs_abi_version() == _lib.ABI_VERSION
    assert torch.cuda.is_available()


def test_homo_warping_seam():
    g = golden("ops.npz")
    p = torch.from_numpy(g["warp_proj"])
    out = ops.homo_warping(torch.from_numpy(g["warp_src"]).to(DEV), oracle.compose_proj(p[:, 1]),
                           oracle.compose_proj(p[:, 0]), torch.from_numpy(g["warp_hyp"]).to(DEV),
                           rot_order=GOLDEN_ROT_ORDER)
    _close(to_np(out), g["warp_out"], 0.0, "homo_warping seam vs golden")


@pytest.mark.parametrize("c,d", [(8, 8), (16, 32), (32, 48)])
def test_warp_corr_stage1_mode(sd, c, d):
    """Fused warp+corr+PixelwiseNet+aggregation vs oracle build_cost_volume (3 src views)."""
    torch.manual_seed(c + d)
    n, h, w = 4, 24, 40
    feats = [torch.randn(1, c, h, w) for _ in range(n)]
    proj = synthetic.synthetic_cameras(n, h * 4, w * 4, seed=5)["stage1"]
    hyp = (torch.rand(1, d, h, w) * 500 + 425)
    hyp[0, 0, :3] = -20.0  # behind camera
    sim_ref, vw_ref = oracle.build_cost_volume(sd, feats, proj, hyp)
    nh = [_nhwc(f).to(DEV) for f in feats]
    src = torch.stack([x[0] for x in nh[1:]], 0).unsqueeze(0).contiguous()
    sim, _, vw = ops.warp_corr(nh[0], src, ops.proj_rows(proj), hyp.to(DEV), pw_params=_pw_params(sd))
    _close(to_np(sim)[:, None], to_np(sim_ref), 5e-7, f"stage1-mode sim c{c} d{d}")
    _close(to_np(vw), to_np(vw_ref), 5e-7, f"stage1-mode view weights c{c} d{d}")


@pytest.mark.parametrize("c,d,stage1", [(32, 48, True), (16, 32, False), (8, 8, False)])
def test_warp_corr_ten_source_views(sd, c, d, stage1):
    """N=11 (configs C3/C4: DTU / Tanks&Temples with 10 source views) through one launch."""
    torch.manual_seed(100 + c)
    n, h, w = 11, 20, 36  # TnT-like aspect
    feats = [torch.randn(1, c, h, w) for _ in range(n)]
    proj = synthetic.synthetic_cameras(n, h * 4, w * 4, seed=9)["stage1"]
    hyp = torch.rand(1, d, h, w) * 500 + 425
    nh = [_nhwc(f).to(DEV) for f in feats]
    src = torch.stack([x[0] for x in nh[1:]], 0).unsqueeze(0).contiguous()
    rows = ops.proj_rows(proj)
    if stage1:
        sim_ref, vw_ref = oracle.build_cost_volume(sd, feats, proj, hyp)
        sim, _, vw = ops.warp_corr(nh[0], src, rows, hyp.to(DEV), pw_params=_pw_params(sd))
        _close(to_np(vw), to_np(vw_ref), 5e-7, f"N=11 view weights c{c}")
    else:
        vw = torch.rand(1, n - 1, h, w)
        sim_ref, _ = oracle.build_cost_volume({}, feats, proj, hyp, view_weights=vw)
        sim, _, _ = ops.warp_corr(nh[0], src, rows, hyp.to(DEV), view_w_in=vw.to(DEV), vw_shift=0)
    _close(to_np(sim)[:, None], to_np(sim_ref), 5e-7, f"N=11 sim c{c}")


@pytest.mark.parametrize("given", [False, True])
def test_warp_corr_dtu_stage1_size(sd, given):
    """Fused cost volume at the DTU stage-1 size (216x288, C=32, D=48, 4 src views) with the
    forward's uniform fronto-parallel planes, against the oracle. 3M outputs: the channel-sum order
    left 5 of them between 2e-5 and 2.7e-5 in round 1, before the host-BLAS rounding of the sample
    coordinates was reproduced; now within 1.1e-7."""
    torch.manual_seed(7)
    n, h, w, c, d = 5, 216, 288, 32, 48
    feats = [torch.randn(1, c, h, w) for _ in range(n)]
    proj = synthetic.synthetic_cameras(n, h * 4, w * 4, seed=1)["stage1"]
    dv = synthetic.synthetic_depth_values(1)
    hyp = oracle.stage_hypotheses(None, dv, 0, (h * 4, w * 4), (48, 32, 8), (4.0, 1.0, 0.5))
    nh = [_nhwc(f).to(DEV) for f in feats]
    src = torch.stack([x[0] for x in nh[1:]], 0).unsqueeze(0).contiguous()
    rows = ops.proj_rows(proj)
    if given:
        vw = torch.rand(1, n - 1, h, w)
        sim_ref, _ = oracle.build_cost_volume({}, feats, proj, hyp, view_weights=vw)
        sim, _, _ = ops.warp_corr(nh[0], src, rows, hyp.to(DEV), view_w_in=vw.to(DEV), vw_shift=0)
    else:
        sim_ref, vw_ref = oracle.build_cost_volume(sd, feats, proj, hyp)
        sim, _, vw_out = ops.warp_corr(nh[0], src, rows, hyp.to(DEV), pw_params=_pw_params(sd))
        _close(to_np(vw_out), to_np(vw_ref), 5e-7, "DTU stage-1 view weights")
    _close(to_np(sim)[:, None], to_np(sim_ref), 5e-7, f"DTU stage-1 sim (given={given})")


def test_warp_corr_incoherent_depth_and_degenerate_planes(sd):
    """C=32 with per-pixel random hypotheses over the whole DTU range, one coherent tile and a
    patch of planes behind the camera (z < 1e-6 -> zero samples), against the oracle."""
    torch.manual_seed(8)
    n, h, w, c, d = 4, 40, 72, 32, 32
    feats = [torch.randn(1, c, h, w) for _ in range(n)]
    proj = synthetic.synthetic_cameras(n, h * 4, w * 4, seed=2)["stage1"]
    hyp = torch.sort(torch.rand(1, d, h, w) * 480 + 425, dim=1).values
    hyp[:, :, :8, :16] = hyp[:, :, :8, :16] * 0 + torch.linspace(600, 640, d).view(1, d, 1, 1)
    hyp[0, 3, 20:24, 30:40] = -30.0
    nh = [_nhwc(f).to(DEV) for f in feats]
    src = torch.stack([x[0] for x in nh[1:]], 0).unsqueeze(0).contiguous()
    sim_ref, vw_ref = oracle.build_cost_volume(sd, feats, proj, hyp)
    sim, _, vw = ops.warp_corr(nh[0], src, ops.proj_rows(proj), hyp.to(DEV), pw_params=_pw_params(sd))
    _close(to_np(sim)[:, None], to_np(sim_ref), 5e-7, "incoherent sim")
    _close(to_np(vw), to_np(vw_ref), 5e-7, "incoherent view weights")


@pytest.mark.parametrize("c,d,interval,scale", [(16, 32, 2.5, "stage2"), (8, 8, 1.25, "stage3"),
                                                (16, 16, 2.5, "stage2"), (8, 64, 1.0, "stage3")])
def test_warp_corr_stage23_segments(c, d, interval, scale):
    """Stages 2/3 (given view weights) with the forward's kind of hypotheses: per pixel D increasing
    planes `interval` mm apart around a random centre, so each pixel-view's taps lie on a short
    epipolar segment (warp_dot_kernel's per-pixel tap window). Mixed in: a patch of pixels whose
    planes span 400 mm (segments longer than the window), a patch with one plane behind the camera,
    and a patch with decreasing planes -- those pixels take the per-lane gather path. Against the
    oracle's build_cost_volume."""
    torch.manual_seed(11 + d)
    n, h, w = 5, 48, 80
    feats = [torch.randn(1, c, h, w) for _ in range(n)]
    mult = 2 if scale == "stage2" else 4
    proj = synthetic.synthetic_cameras(n, h * 4 // mult, w * 4 // mult, seed=2)[scale]
    centre = torch.rand(1, 1, h, w) * 450 + 450
    hyp = centre + (torch.arange(d, dtype=torch.float32) - d / 2).view(1, d, 1, 1) * interval
    hyp[:, :, 4:10, 4:20] = torch.linspace(450.0, 850.0, d).view(1, d, 1, 1)
    hyp[0, d // 2, 20:24, 30:40] = -30.0
    hyp[:, :, 30:36, 50:70] = hyp[:, :, 30:36, 50:70].flip(1)
    vw = torch.rand(1, n - 1, h, w)
    sim_ref, _ = oracle.build_cost_volume({}, feats, proj, hyp, view_weights=vw)
    nh = [_nhwc(f).to(DEV) for f in feats]
    src = torch.stack([x[0] for x in nh[1:]], 0).unsqueeze(0).contiguous()
    sim, _, _ = ops.warp_corr(nh[0], src, ops.proj_rows(proj), hyp.to(DEV), view_w_in=vw.to(DEV), vw_shift=0)
    _close(to_np(sim)[:, None], to_np(sim_ref), 5e-7, f"segments c{c} d{d}")


def test_e2e_eleven_views_tnt_aspect(sd):
    """Whole hot path at N=11 on a Tanks&Temples-shaped (1056x1920 / 4) frame vs the oracle."""
    m = TransMVSNet().eval()
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    H, W, N = 256, 480, 11
    feats = synthetic.synthetic_features(N, H, W, seed=4)
    proj = synthetic.synthetic_cameras(N, H, W, seed=3)
    dv = synthetic.synthetic_depth_values(1)
    ref = oracle.forward_from_features(sd, feats, proj, dv, (H, W))
    with torch.no_grad():
        out = m.forward_features([{k: v.to(DEV) for k, v in f.items()} for f in feats], proj, dv.to(DEV), (H, W))
    for s in (1, 2, 3):
        mean_l1, near, flips = depth_parity(to_np(out[f"stage{s}"]["depth"]), to_np(ref[f"stage{s}"]["depth"]),
                                            to_np(ref[f"stage{s}"]["prob_volume"]))
        assert flips == 0, (s, mean_l1, near, flips)
    l1 = float(np.abs(to_np(out["depth"]).astype(np.float64) - to_np(ref["depth"]).astype(np.float64)).mean())
    assert l1 <= 1e-4, l1


def _pw_params(sd):
    m = TransMVSNet()
    m.load_state_dict(sd, strict=True)
    return m.DepthNet.pixel_wise_net.packed()


@pytest.mark.parametrize("shift", [1, 2])
def test_warp_corr_given_weights_and_partial(shift):
    torch.manual_seed(shift)
    n, h, w, c, d = 5, 32, 48, 8, 8
    feats = [torch.randn(1, c, h, w) for _ in range(n)]
    proj = synthetic.synthetic_cameras(n, h, w, seed=6)["stage3"]
    hyp = torch.rand(1, d, h, w) * 500 + 425
    vw = torch.rand(1, n - 1, h >> shift, w >> shift)
    vw_up = vw
    for _ in range(shift):
        vw_up = F.interpolate(vw_up, scale_factor=2, mode="nearest")
    sim_ref, _ = oracle.build_cost_volume({}, feats, proj, hyp, view_weights=vw_up)
    nh = [_nhwc(f).to(DEV) for f in feats]
    src = torch.stack([x[0] for x in nh[1:]], 0).unsqueeze(0).contiguous()
    rows = ops.proj_rows(proj)
    sim, _, _ = ops.warp_corr(nh[0], src, rows, hyp.to(DEV), view_w_in=vw.to(DEV), vw_shift=shift)
    _close(to_np(sim)[:, None], to_np(sim_ref), 5e-7, f"given weights shift{shift}")
    # view-sharded form: two partial sums (views 0-1 and 2-3) + finalize == unsharded
    s_a, w_a, _ = ops.warp_corr(nh[0], src[:, :2].contiguous(), rows[:, :2], hyp.to(DEV), view_w_in=vw.to(DEV),
                                vw_shift=shift, vw_offset=0, vw_total=4, partial=True)
    s_b, w_b, _ = ops.warp_corr(nh[0], src[:, 2:].contiguous(), rows[:, 2:], hyp.to(DEV), view_w_in=vw.to(DEV),
                                vw_shift=shift, vw_offset=2, vw_total=4, partial=True)
    fin = ops.aggregate_finalize(s_a + s_b, w_a + w_b)
    np.testing.assert_allclose(to_np(fin), to_np(sim), rtol=0, atol=2e-6)


def test_costregnet_matches_golden(model):
    g = golden("ops.npz")
    x = torch.from_numpy(g["costreg_in"])[:, 0].to(DEV).contiguous()
    st, _keep = model.cost_regularization[0].packed(DEV)
    out = to_np(ops.costregnet(x, st))
    ref = g["costreg_out"][:, 0]
    scale = np.abs(ref).max()
    assert np.abs(out - ref).max() <= 2e-5 * scale, (np.abs(out - ref).max(), scale)


@pytest.mark.parametrize("layer,stride", [("conv1", 2), ("conv2", 1), ("conv3", 2), ("conv4", 1), ("conv5", 2),
                                          ("conv6", 1)])
def test_conv3d_layers(sd, model, layer, stride):
    blk = getattr(model.cost_regularization[1], layer)
    w = blk.conv.weight.detach().cpu()
    co, ci = w.shape[:2]
    x = torch.randn(1, ci, 8, 12, 20)
    p = f"cost_regularization.1.{layer}."
    ref = F.relu(F.batch_norm(F.conv3d(x, w, stride=stride, padding=1), sd[p + "bn.running_mean"],
                              sd[p + "bn.running_var"], sd[p + "bn.weight"], sd[p + "bn.bias"], False, 0.1, 1e-5))
    st, keep = model.cost_regularization[1].packed(DEV)
    idx = int(layer[4:])
    xin = x.permute(0, 2, 3, 4, 1).contiguous().to(DEV)
    y = ops.conv3d_bn_relu(xin, keep[idx], keep[11 + idx], keep[21 + idx], co, stride)
    np.testing.assert_allclose(to_np(y), ref.permute(0, 2, 3, 4, 1).numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("layer,idx", [("conv7", 7), ("conv9", 8), ("conv11", 9)])
def test_deconv3d_layers(sd, model, layer, idx):
    blk = getattr(model.cost_regularization[1], layer)
    w = blk.conv.weight.detach().cpu()
    ci, co = w.shape[:2]
    x = torch.randn(1, ci, 4, 6, 10)
    skip = torch.randn(1, co, 8, 12, 20)
    p = f"cost_regularization.1.{layer}."
    y_ref = skip + F.relu(F.batch_norm(F.conv_transpose3d(x, w, stride=2, padding=1, output_padding=1),
                                       sd[p + "bn.running_mean"], sd[p + "bn.running_var"], sd[p + "bn.weight"],
                                       sd[p + "bn.bias"], False, 0.1, 1e-5))
    st, keep = model.cost_regularization[1].packed(DEV)
    y = ops.deconv3d_bn_relu_add(x.permute(0, 2, 3, 4, 1).contiguous().to(DEV), keep[idx], keep[11 + idx],
                                 keep[21 + idx], co, skip.permute(0, 2, 3, 4, 1).contiguous().to(DEV))
    np.testing.assert_allclose(to_np(y), y_ref.permute(0, 2, 3, 4, 1).numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("d,h,w,b", [(8, 232, 264, 2), (8, 16, 40, 1), (32, 232, 264, 2), (48, 24, 32, 2),
                                     (64, 16, 72, 1), (16, 40, 128, 1), (24, 8, 8, 2), (32, 432, 576, 1),
                                     (8, 864, 1152, 1)])
def test_costregnet_wta_equals_costregnet_then_softmax(model, d, h, w, b):
    """tmvs_costregnet_wta (prob conv + softmax/WTA in one kernel for D <= 32; the depth-chunked
    prob kernel + softmax kernel for 48/64) == tmvs_costregnet -> tmvs_softmax_wta, bit for bit (ragged
    shapes, tiny volumes, B = 2 and the DTU stage-2/3 sizes)."""
    g = torch.Generator().manual_seed(d * 1000 + h)
    x = torch.randn(b, d, h, w, generator=g).to(DEV)
    hyp = (425.0 + torch.rand(b, d, h, w, generator=g).mul(510.0)).sort(dim=1).values.to(DEV)
    st, _keep = model.cost_regularization[1].packed(DEV)
    ref = ops.softmax_wta(ops.costregnet(x, st), hyp, (500.0, 900.0))
    got = ops.costregnet_wta(x, st, hyp, (500.0, 900.0))
    for name, a, r in zip(("prob", "depth", "depth_raw", "conf"), got, ref):
        np.testing.assert_array_equal(to_np(a), to_np(r), err_msg=name)


def test_softmax_wta_ties():
    g = golden("ops.npz")
    prob, depth, raw, conf = ops.softmax_wta(torch.from_numpy(g["wta_logits"]).to(DEV),
                                             torch.from_numpy(g["wta_hyp"]).to(DEV), clamp=(-1e30, 1e30))
    np.testing.assert_allclose(to_np(prob), g["wta_prob"], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(to_np(depth), g["wta_depth"])
    np.testing.assert_allclose(to_np(conf), g["wta_conf"], rtol=0, atol=1e-6)


def test_stage_hypotheses_bitexact():
    g = golden("ops.npz")
    dv = synthetic.synthetic_depth_values(1).to(DEV)
    h2 = ops.stage_hypotheses(dv, torch.from_numpy(g["glue2_prev"]).to(DEV), 32, 1.0, (64, 80), 2)
    np.testing.assert_array_equal(to_np(h2), g["glue2_hyp"])
    h3 = ops.stage_hypotheses(dv, torch.from_numpy(g["glue3_prev"]).to(DEV), 8, 0.5, (64, 80), 1)
    np.testing.assert_array_equal(to_np(h3), g["glue3_hyp"])
    h1 = ops.stage_hypotheses(dv, None, 48, 4.0, (64, 80), 4)
    ref = oracle.stage_hypotheses(None, synthetic.synthetic_depth_values(1), 0, (64, 80))
    np.testing.assert_array_equal(to_np(h1), ref.numpy())


def test_fmt_encoder_layer(model):
    g = golden("ops.npz")
    enc = model.FMT_with_pathway.FMT.layers[1].packed().to(DEV)
    x = torch.from_numpy(g["enc_x"]).to(DEV).contiguous()
    src = torch.from_numpy(g["enc_src"]).to(DEV).contiguous()
    kv = ops.fmt_kv(src, enc)
    ops.fmt_apply(x, kv, enc)
    _close(to_np(x), g["enc_out"], 2e-6, "EncoderLayer vs golden")


# the two-stream FMT (reference chain on a side stream) against the one-stream orchestration, bit for bit,
# at a ragged token count and at the DTU stage-1 size whose K/V launches use 8 tiles per wave; and the
# grouped K/V of view subsets against the batched launch
@pytest.mark.parametrize("nv,h,w", [(3, 37, 53), (5, 216, 288)])
def test_fmt_forward_split_bitwise(model, nv, h, w):
    torch.manual_seed(11)
    prep = model._prepared(torch.device(DEV))
    s1 = torch.randn(nv, 32, h, w, device=DEV)
    pe = model._pe_slice(h, w, torch.device(DEV))
    ref = ops.fmt_forward(s1, pe, prep["enc"])
    side = torch.cuda.Stream(torch.device(DEV))
    for _ in range(2):
        out = ops.fmt_forward(s1, pe, prep["enc"], side_stream=side)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), "split FMT differs from the one-stream FMT"
    lib = _lib.load()
    L = h * w
    kv_all = ops.fmt_kv(ref, prep["enc"][2])
    for lo, hi in ((0, 1), (1, nv)):
        kv = torch.empty(hi - lo, _lib.KV_NFLOATS, device=DEV)
        nbytes = lib.tmvs_fmt_kv_grouped_workspace(hi - lo, nv, L)
        ws = torch.empty(nbytes // 4 + 1, device=DEV)
        _lib.check(lib.tmvs_fmt_kv_grouped(ref[lo:hi].data_ptr(), hi - lo, nv, L, prep["enc"][2].data_ptr(),
                                           ws.data_ptr(), ws.numel() * 4, kv.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream), "kv_grouped")
        torch.cuda.synchronize()
        assert torch.equal(kv, kv_all[lo:hi]), f"grouped K/V views {lo}..{hi}"


# (views, coarse h, w): one partial tile row; ragged tiles over 798 tiles, i.e. runs of 2 tiles per
# workgroup of the pipelined stage-2 kernel with a short last run
@pytest.mark.parametrize("nv,h,w", [(2, 12, 20), (3, 109, 147)])
def test_fmt_pathway(sd, model, nv, h, w):
    torch.manual_seed(3)
    coarse = torch.randn(nv, 32, h, w)
    lat = torch.randn(nv, 16, 2 * h, 2 * w)
    ref = F.conv2d(F.interpolate(F.conv2d(coarse, sd["FMT_with_pathway.dim_reduction_1.weight"]), size=(2 * h, 2 * w),
                                 mode="bilinear") + lat, sd["FMT_with_pathway.smooth_1.weight"], padding=1)
    prep = model._prepared(torch.device(DEV))
    out = ops.fmt_pathway(coarse.permute(0, 2, 3, 1).contiguous().to(DEV), lat.to(DEV), prep["red1"], prep["sm1"])
    _close(to_np(out), ref.permute(0, 2, 3, 1).numpy(), 3e-6, "pathway")


def _e2e_check(out, vw, g, stages=(1, 2, 3)):
    report = {}
    for s in stages:
        o = out[f"stage{s}"]
        pref = g.get(f"stage{s}_prob")
        if pref is not None:
            mean_l1, near, flips = depth_parity(to_np(o["depth"]), g[f"stage{s}_depth"], pref)
            if s == 1:
                np.testing.assert_array_equal(to_np(o["depth_values"]), g[f"stage{s}_hyp"])
            report[s] = (mean_l1, near, flips)
            assert flips == 0, (s, report[s])
        mean_l1 = float(np.abs(to_np(o["depth"]).astype(np.float64) - g[f"stage{s}_depth"]).mean())
        report[f"l1_{s}"] = mean_l1
    assert report["l1_3"] <= 1e-4, report
    if vw is not None:
        _close(to_np(vw), g["view_weights"], 5e-7, "e2e view weights vs golden")
    return report


def test_e2e_c1_features(model):
    g = golden("e2e_c1_features.npz")
    H, W, N = 128, 160, 3
    feats = [{k: v.to(DEV) for k, v in f.items()} for f in synthetic.synthetic_features(N, H, W, seed=2)]
    with golden_rot(model):
        out, vw = model.forward_features(feats, synthetic.synthetic_cameras(N, H, W, seed=1),
                                         synthetic.synthetic_depth_values(1).to(DEV), (H, W), return_view_weights=True)
    rep = _e2e_check(out, vw, g)
    for s in (1, 2, 3):
        _close(to_np(out[f"stage{s}"]["prob_volume"]), g[f"stage{s}_prob"], 2e-4, f"e2e C1 prob stage{s}")
    print("e2e c1", rep)


def test_e2e_cascade_48_32_8(sd):
    g = golden("e2e_cascade_256x320.npz")
    m = TransMVSNet().eval()
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    m.warp_rot_order = GOLDEN_ROT_ORDER
    H, W, N = 256, 320, 3
    feats = [{k: v.to(DEV) for k, v in f.items()} for f in synthetic.synthetic_features(N, H, W, seed=2)]
    out, vw = m.forward_features(feats, synthetic.synthetic_cameras(N, H, W, seed=1),
                                 synthetic.synthetic_depth_values(1).to(DEV), (H, W), return_view_weights=True)
    print("e2e cascade", _e2e_check(out, vw, g))


def test_e2e_hip_graph_replay_is_bitwise_eager(sd):
    """bench.py's step as one captured HIP graph (FMT, the pathway's side stream, 3 stages) replays
    to exactly the eager forward's outputs, also after the inputs are overwritten in place."""
    m = TransMVSNet().eval()
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    H, W, N = 256, 320, 3
    feats = synthetic.stacked_features(N, H, W, seed=2)
    feats = {k: v.to(DEV) for k, v in feats.items()}
    proj = synthetic.synthetic_cameras(N, H, W, seed=1)
    dv = synthetic.synthetic_depth_values(1).to(DEV)
    with torch.no_grad():
        ref = m.forward_features(feats, proj, dv, (H, W))
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = m.forward_features(feats, proj, dv, (H, W))
        graph.replay()
        torch.cuda.synchronize()
        for s in (1, 2, 3):
            for k in ("depth", "prob_volume", "photo_confidence"):
                assert torch.equal(out[f"stage{s}"][k], ref[f"stage{s}"][k]), (s, k)
        feats2 = synthetic.stacked_features(N, H, W, seed=7)
        for k in feats:
            feats[k].copy_(feats2[k].to(DEV))
        ref2 = m.forward_features(feats, proj, dv, (H, W))
        graph.replay()
        torch.cuda.synchronize()
        assert not torch.equal(ref2["stage3"]["depth"], ref["stage3"]["depth"])
        for s in (1, 2, 3):
            assert torch.equal(out[f"stage{s}"]["depth"], ref2[f"stage{s}"]["depth"]), s


def test_e2e_cascade_view_sharded_path(sd):
    """transmvsnet_amd.distributed on one rank: partial cost volume + finalize + replicated CostRegNet."""
    from transmvsnet_amd.distributed import ViewShard
    g = golden("e2e_cascade_256x320.npz")
    m = TransMVSNet().eval()
    m.load_state_dict(sd, strict=True)
    m = m.to(DEV)
    m.warp_rot_order = GOLDEN_ROT_ORDER
    H, W, N = 256, 320, 3
    feats = [{k: v.to(DEV) for k, v in f.items()} for f in synthetic.synthetic_features(N, H, W, seed=2)]
    out, vw = m.forward_features(feats, synthetic.synthetic_cameras(N, H, W, seed=1),
                                 synthetic.synthetic_depth_values(1).to(DEV), (H, W), return_view_weights=True,
                                 view_shard=ViewShard(0, 1, N - 1))
    print("e2e cascade (view-sharded path)", _e2e_check(out, vw, g))


def test_e2e_images_full_forward(model):
    g = golden("e2e_c1_imgs.npz")
    H, W, N = 128, 160, 3
    with torch.no_grad(), golden_rot(model):
        out = model(synthetic.synthetic_images(N, H, W, seed=0).to(DEV), synthetic.synthetic_cameras(N, H, W, seed=1),
                    synthetic.synthetic_depth_values(1).to(DEV))
    l1 = float(np.abs(to_np(out["depth"]).astype(np.float64) - g["stage3_depth"]).mean())
    assert l1 <= 1e-4, l1
    assert set(out) == {"stage1", "stage2", "stage3", "depth", "photo_confidence", "prob_volume", "depth_values"}


def test_e2e_images_batch_of_two(sd, model):
    """forward() on a batch of 2 different samples (FeatureNet batches all B*N views; the hot path
    loops over B): each sample's outputs equal the oracle's single-sample forward."""
    from oracle import transmvs_ref as oracle
    H, W, N = 64, 96, 3
    imgs = torch.cat([synthetic.synthetic_images(N, H, W, seed=10), synthetic.synthetic_images(N, H, W, seed=11)], 0)
    cams = [synthetic.synthetic_cameras(N, H, W, seed=20), synthetic.synthetic_cameras(N, H, W, seed=21)]
    proj = {k: torch.cat([c[k] for c in cams], 0) for k in cams[0]}
    dv = torch.cat([synthetic.synthetic_depth_values(1), synthetic.synthetic_depth_values(1) + 5.0], 0)
    with torch.no_grad():
        out = model(imgs.to(DEV), proj, dv.to(DEV))
        for b in range(2):
            ref = oracle.forward(sd, imgs[b:b + 1], {k: v[b:b + 1] for k, v in proj.items()}, dv[b:b + 1],
                                 ndepths=(8, 8, 8))
            d = np.abs(to_np(out["depth"][b]).astype(np.float64) - ref["depth"][0].numpy()).mean()
            assert d <= 1e-4, (b, d)
            np.testing.assert_allclose(to_np(out["stage1"]["prob_volume"][b]), to_np(ref["stage1"]["prob_volume"][0]),
                                       atol=1e-5)
    assert out["depth"].shape == (2, H, W) and out["prob_volume"].shape == (2, 8, H, W)


def test_e2e_images_batch_of_two_different_depth_ranges(sd, model):
    """B=2 whose samples have different depth-range widths, against the oracle's BATCHED forward:
    stage 1 samples each sample's own range, stages 2/3 take the hypothesis interval from
    depth_values[0] for both samples (models/TransMVSNet.py:146-148, get_depth_samples)."""
    from oracle import transmvs_ref as oracle
    H, W, N = 64, 96, 3
    imgs = torch.cat([synthetic.synthetic_images(N, H, W, seed=12), synthetic.synthetic_images(N, H, W, seed=13)], 0)
    cams = [synthetic.synthetic_cameras(N, H, W, seed=22), synthetic.synthetic_cameras(N, H, W, seed=23)]
    proj = {k: torch.cat([c[k] for c in cams], 0) for k in cams[0]}
    dv0 = synthetic.synthetic_depth_values(1)
    dv = torch.cat([dv0, 450.0 + (dv0 - 425.0) * 1.5], 0)   # sample 1: 450..1166 mm, 1.5x the interval
    with torch.no_grad():
        out = model(imgs.to(DEV), proj, dv.to(DEV))
        ref = oracle.forward(sd, imgs, proj, dv, ndepths=(8, 8, 8))
    for s in (1, 2, 3):
        dh = np.abs(to_np(out[f"stage{s}"]["depth_values"]) - to_np(ref[f"stage{s}"]["depth_values"]))
        # bit-exact where the previous stage's depth agrees (a near-tie flip upstream moves a few pixels)
        assert (dh.max() == 0) if s == 1 else (np.median(dh) == 0 and (dh > 0).mean() < 0.01), (s, dh.max())
        mean_l1, near, flips = depth_parity(to_np(out[f"stage{s}"]["depth"]), to_np(ref[f"stage{s}"]["depth"]),
                                            to_np(ref[f"stage{s}"]["prob_volume"]))
        assert flips == 0, (s, mean_l1, near, flips)


def test_batch_samples_on_concurrent_streams_bitwise(model):
    """B = 3 from features with the samples on concurrent streams (model.batch_streams, the default) is
    bitwise the sequential per-sample form (batch_streams False) and each sample's single-sample forward;
    a HIP-graph capture of the B = 3 step (samples in order on the capturing stream) replays the same bits."""
    H, W, N = 64, 96, 3
    fs = [synthetic.synthetic_features(N, H, W, seed=30 + b) for b in range(3)]
    feats = {k: torch.cat([model.stack_features(f)[k] for f in fs], 0).to(DEV) for k in ("stage1", "stage2", "stage3")}
    cams = [synthetic.synthetic_cameras(N, H, W, seed=40 + b) for b in range(3)]
    proj = {k: torch.cat([c[k] for c in cams], 0) for k in cams[0]}
    dv = torch.cat([synthetic.synthetic_depth_values(1) + 3.0 * b for b in range(3)], 0).to(DEV)
    keys = ("depth", "photo_confidence", "prob_volume", "depth_values")
    with torch.no_grad():
        model.batch_streams = False
        try:
            seq = model.forward_features(feats, proj, dv, (H, W))
        finally:
            model.batch_streams = True
        con = model.forward_features(feats, proj, dv, (H, W))
        # sample 0 alone (later samples take stages 2/3's interval from depth_values[0] in a batch)
        one = model.forward_features({k: v[0:1] for k, v in feats.items()}, {k: v[0:1] for k, v in proj.items()},
                                     dv[0:1], (H, W))
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_out = model.forward_features(feats, proj, dv, (H, W))
        graph.replay()
        torch.cuda.synchronize()
    for s in (1, 2, 3):
        for k in keys:
            a, c, r = seq[f"stage{s}"][k], con[f"stage{s}"][k], g_out[f"stage{s}"][k]
            assert torch.equal(a, c), (s, k)
            assert torch.equal(a, r), (s, k, "graph")
            assert torch.equal(a[0:1], one[f"stage{s}"][k]), (s, k, "single")
