"""CostRegNet training on the GPU: transmvsnet_amd.train's
train-mode forward + HIP backward against torch autograd through the oracle's CostRegNet in train
mode (models/module.py:447-456 with BatchNorm3d batch statistics), at a small shape and the three
C5 stage shapes (BlendedMVS 768x576: 48 x 144x192, 32 x 288x384, 8 x 576x768).

The reference is evaluated twice on the CPU: in fp32 (what the reference computes) and in fp64
(the exact value). At the C5 sizes the fp32 reference's own gradients are 0.5-1.2 % (of their max
magnitude) away from the fp64 ones (BatchNorm's backward subtracts batch means of 1e5-1e6 terms;
measured: dx 4.7e-3 at 48x144x192, 1.2e-2 at 8x576x768), so the gradients are judged against fp64:
  logits: 1e-4 of max|logits| against the fp32 reference;
  every gradient (dx, each weight / gamma / beta): error against fp64 <= max(1e-4, twice the fp32
  reference's own error on that gradient, the fp32 reference's worst error over all of this
  network's gradients at this size), all relative to the quantity's max magnitude;
  running statistics: 1e-5 of their max magnitude.
"""
import numpy as np
import pytest
import torch

from oracle import transmvs_ref as oracle
from tests._util import golden_state_dict
from transmvsnet_amd.model import CostRegNet
from transmvsnet_amd.train import costregnet_params, costregnet_train

pytestmark = pytest.mark.gpu
DEV = "cuda"
PREFIX = "cost_regularization.0."


def _rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


@pytest.mark.parametrize("shape", [(1, 8, 32, 40), (2, 8, 16, 24), (1, 48, 144, 192), (1, 32, 288, 384),
                                   (1, 8, 576, 768)])
def test_costregnet_train_forward_backward(shape):
    sd = {k[len(PREFIX):]: v for k, v in golden_state_dict().items() if k.startswith(PREFIX)}
    cr = CostRegNet(1, 8)
    cr.load_state_dict(sd, strict=True)
    cr = cr.to(DEV).train()
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(shape, generator=g) * 0.5
    gout = torch.randn(shape, generator=g)
    xg = x.to(DEV).requires_grad_()
    out = costregnet_train(cr, xg)
    out.backward(gout.to(DEV))
    torch.cuda.synchronize()
    # reference: torch autograd through the oracle in train mode (CPU), fp32 and fp64
    refs = {}
    for dt in (torch.float32, torch.float64):
        r_sd = {k: (v.to(dt).clone().requires_grad_() if v.is_floating_point() and "running" not in k
                    else (v.to(dt).clone() if v.is_floating_point() else v.clone())) for k, v in sd.items()}
        xc = x.to(dt).clone().requires_grad_()
        r = oracle.cost_reg_net(r_sd, "", xc.unsqueeze(1), training=True)[:, 0]
        r.backward(gout.to(dt))
        refs[dt] = (r, xc.grad, r_sd)
    ref, ref_dx, ref_sd = refs[torch.float32]
    ex, ex_dx, ex_sd = refs[torch.float64]
    rep = {"logits": _rel(out, ref)}
    assert rep["logits"] < 1e-4, rep
    names = [n for n in sd if n.endswith(("conv.weight", "bn.weight", "bn.bias"))] + ["prob.weight"]
    params = dict(zip([f"{n}.{s}" for n in ("conv0", "conv1", "conv2", "conv3", "conv4", "conv5", "conv6", "conv7",
                                             "conv9", "conv11") for s in ("conv.weight", "bn.weight", "bn.bias")]
                      + ["prob.weight"], costregnet_params(cr)))
    assert set(params) == set(names)
    checks = [("dx", xg.grad, ref_dx, ex_dx)] + [(n, params[n].grad, ref_sd[n].grad, ex_sd[n].grad) for n in names]
    worst = (0.0, None, 0.0)
    errs = [(n, _rel(got, r64), _rel(r32, r64)) for n, got, r32, r64 in checks]
    ref_worst = max(e for _, _, e in errs)
    print(shape, "gradient errors vs fp64 (name, gpu, fp32 reference):",
          [(n, f"{a:.1e}", f"{b:.1e}") for n, a, b in errs])
    for n, e_gpu, e_ref in errs:
        assert e_gpu <= max(1e-4, 2.0 * e_ref, ref_worst), (n, e_gpu, e_ref, ref_worst)
        worst = max(worst, (e_gpu, n, e_ref))
    rep["worst_grad_vs_fp64 (gpu, name, fp32 reference)"] = worst
    rep["dx_vs_fp64 (gpu, fp32 reference)"] = (_rel(xg.grad, ex_dx), _rel(ref_dx, ex_dx))
    for n in sd:
        if "running" in n:
            r = _rel(dict(cr.named_buffers())[n], ref_sd[n])
            assert r < 1e-5, (n, r)
    assert int(cr.conv0.bn.num_batches_tracked) == 1 + int(sd["conv0.bn.num_batches_tracked"])
    print(shape, rep)


@pytest.mark.parametrize("cin,cout,stride,transposed", [(16, 16, 1, False), (32, 32, 1, False), (64, 64, 1, False),
                                                         (8, 16, 2, False), (16, 32, 2, False), (32, 64, 2, False),
                                                         (64, 32, 2, True), (32, 16, 2, True), (16, 8, 2, True),
                                                         (1, 8, 1, False), (8, 1, 1, False)])
@pytest.mark.parametrize("dims", [(4, 10, 20), (1, 6, 37)])
def test_conv3d_mfma_raw_vs_torch(cin, cout, stride, transposed, dims):
    """tmvs_conv3d_mfma (the inference layers' MFMA kernels, and conv0's / prob's VALU kernels, with the
    raw epilogue) against torch's
    fp32 conv3d / conv_transpose3d (k3 p1, op1), incl. ragged H/W and depth 1, negative outputs kept
    (no ReLU) and the transposed form's skip add. Bar: 2e-6 of max|y| (K = 27 cin fp32 terms)."""
    import torch.nn.functional as F
    from transmvsnet_amd import ops
    from transmvsnet_amd.train import _pack_fwd
    torch.manual_seed(cin + cout + dims[2])
    x = torch.randn(1, cin, *dims)
    w = torch.randn(*((cin, cout) if transposed else (cout, cin)), 3, 3, 3) * 0.1
    if transposed:
        ref = F.conv_transpose3d(x, w, stride=2, padding=1, output_padding=1)
        skip = torch.randn(ref.shape)
        ref = ref + skip
    else:
        ref = F.conv3d(x, w, stride=stride, padding=1)
        skip = None
    pk = _pack_fwd(w, transposed)
    if (cin, cout) == (8, 1):
        pk = ops.prob_pack(pk)
    got = ops.conv3d_mfma(x.permute(0, 2, 3, 4, 1).contiguous().to(DEV), pk.to(DEV), cout,
                          stride, transposed,
                          skip=None if skip is None else skip.permute(0, 2, 3, 4, 1).contiguous().to(DEV))
    got = got.permute(0, 4, 1, 2, 3).cpu()
    assert got.shape == ref.shape
    assert float(got.min()) < 0.0
    err = float((got - ref).abs().max()) / float(ref.abs().max())
    assert err < 2e-6, err


@pytest.mark.parametrize("c,d,h,w,nv,scale", [(8, 8, 24, 32, 3, 1.0), (32, 48, 144, 192, 3, 1.0),
                                              (16, 32, 288, 384, 3, 1.0), (8, 8, 576, 768, 3, 1.0),
                                              (8, 8, 576, 768, 3, 1e-9), (32, 48, 144, 192, 3, 1e-7)])
def test_warp_corr_views_forward_backward(c, d, h, w, nv, scale):
    """Per-view similarity volumes + their backward into the reference and source features against
    torch autograd through the oracle's homo_warping + mean (CPU fp32; fp32 relative precision does
    not depend on the scale). The source-feature gradient is a bilinear scatter: the GPU sums it in
    fixed point (deterministic) with the unit chosen per call from max|dsim| * max|ref|. `scale` shrinks dsim to the size a
    mean loss over a full C5 stage produces (d loss / d sim ~ 1e-7..1e-9 per element): an absolute
    fixed-point unit (2^-40) would lose most of those bits."""
    from transmvsnet_amd import ops, synthetic
    from transmvsnet_amd.train import warp_corr_views
    g = torch.Generator().manual_seed(c + d + h)
    feats = [torch.randn(1, c, h, w, generator=g) for _ in range(nv + 1)]
    proj = synthetic.synthetic_cameras(nv + 1, h * (4 if c == 32 else 2 if c == 16 else 1),
                                       w * (4 if c == 32 else 2 if c == 16 else 1), seed=3)
    proj = proj["stage1" if c == 32 else "stage2" if c == 16 else "stage3"]
    hyp = (560.0 + 120.0 * torch.rand(1, d, h, w, generator=g)).contiguous()
    dsim = torch.randn(nv, d, h, w, generator=g) * scale
    rows = ops.proj_rows(proj)[0]
    ref_g = feats[0][0].permute(1, 2, 0).contiguous().to(DEV).requires_grad_()
    src_g = torch.stack([f[0].permute(1, 2, 0) for f in feats[1:]]).contiguous().to(DEV).requires_grad_()
    sims = warp_corr_views(ref_g, src_g, hyp[0].to(DEV), rows)
    sims.backward(dsim.to(DEV))
    torch.cuda.synchronize()
    xs = [f.clone().requires_grad_() for f in feats]
    projs = torch.unbind(proj, 1)
    ref_sims = []
    for i in range(nv):
        warped = oracle.homo_warping(xs[1 + i], oracle.compose_proj(projs[1 + i]), oracle.compose_proj(projs[0]), hyp)
        ref_sims.append((warped * xs[0].unsqueeze(2)).mean(1))
    ref_sims = torch.cat(ref_sims, 0)
    ref_sims.backward(dsim)
    rep = {"sim": float((sims.cpu() - ref_sims).abs().max()),
           "dref": _rel(ref_g.grad.permute(2, 0, 1), xs[0].grad[0]),
           "dsrc": max(_rel(src_g.grad[i].permute(2, 0, 1), xs[1 + i].grad[0]) for i in range(nv))}
    print((c, d, h, w, nv, scale), rep)
    assert rep["sim"] < 2e-5 and rep["dref"] < 1e-5 and rep["dsrc"] < 1e-5, rep


@pytest.mark.parametrize("c,d,h,w,nv,scale,zoom", [(32, 48, 144, 192, 3, 1.0, False), (8, 8, 24, 32, 3, 1.0, False),
                                                   (32, 48, 144, 192, 3, 1e-7, False), (16, 32, 288, 384, 3, 1.0, False),
                                                   (32, 48, 144, 192, 3, 1.0, True), (32, 16, 61, 83, 2, 1.0, True)])
def test_warp_corr_views_backward_planes(c, d, h, w, nv, scale, zoom):
    """The stage-1 backward with fronto-parallel depth planes (TMVS_WARP_BWD_PLANES: d src gathered per
    source texel from the preimage of its tap square under the plane homography, no atomics) against
    torch autograd through the oracle (CPU fp32), and against the fixed-point scatter of the same
    call without the flag. zoom: source views with 2x and 0.5x focal lengths (a preimage box of
    ~1 and ~4 pixels per side) and planes from 300 mm, partly off-image."""
    from transmvsnet_amd import ops, synthetic
    from transmvsnet_amd.train import warp_corr_views
    g = torch.Generator().manual_seed(c + d + h + int(zoom))
    feats = [torch.randn(1, c, h, w, generator=g) for _ in range(nv + 1)]
    proj = synthetic.synthetic_cameras(nv + 1, h * 4, w * 4, seed=3)["stage1"].clone()
    lo = 425.0
    if zoom:
        for v, f in ((1, 2.0), (2, 0.5)):
            proj[0, v, 1, 0, 0] *= f
            proj[0, v, 1, 1, 1] *= f
        lo = 300.0
    hyp = torch.linspace(lo, 935.0, d).view(1, d, 1, 1).expand(1, d, h, w).contiguous()
    dsim = torch.randn(nv, d, h, w, generator=g) * scale
    rows = ops.proj_rows(proj)[0]
    grads = {}
    for planes in (True, False):
        ref_g = feats[0][0].permute(1, 2, 0).contiguous().to(DEV).requires_grad_()
        src_g = torch.stack([f[0].permute(1, 2, 0) for f in feats[1:]]).contiguous().to(DEV).requires_grad_()
        sims = warp_corr_views(ref_g, src_g, hyp[0].to(DEV), rows, planes=planes)
        sims.backward(dsim.to(DEV))
        torch.cuda.synchronize()
        grads[planes] = (ref_g.grad.cpu(), src_g.grad.cpu())
    xs = [f.clone().requires_grad_() for f in feats]
    projs = torch.unbind(proj, 1)
    ref_sims = []
    for i in range(nv):
        warped = oracle.homo_warping(xs[1 + i], oracle.compose_proj(projs[1 + i]), oracle.compose_proj(projs[0]), hyp)
        ref_sims.append((warped * xs[0].unsqueeze(2)).mean(1))
    torch.cat(ref_sims, 0).backward(dsim)
    dref, dsrc = grads[True]
    rep = {"dref": _rel(dref.permute(2, 0, 1), xs[0].grad[0]),
           "dsrc": max(_rel(dsrc[i].permute(2, 0, 1), xs[1 + i].grad[0]) for i in range(nv)),
           "dsrc_vs_scatter": max(_rel(dsrc[i], grads[False][1][i]) for i in range(nv)),
           "dref_vs_scatter": float((dref - grads[False][0]).abs().max())}
    print((c, d, h, w, nv, scale, zoom), rep)
    assert rep["dref"] < 1e-5 and rep["dsrc"] < 1e-5 and rep["dsrc_vs_scatter"] < 1e-5, rep
    assert rep["dref_vs_scatter"] == 0.0, rep  # the same gather kernel (without its scatter half)


def test_warp_corr_backward_planes_flags_nonplanar():
    """planes=True on hypotheses that are not one depth per plane sets flag bit 2 (the backward raises)."""
    from transmvsnet_amd import ops, synthetic
    c, d, h, w, nv = 8, 8, 24, 32, 2
    g = torch.Generator().manual_seed(5)
    ref = torch.randn(h, w, c, generator=g).to(DEV)
    src = torch.randn(nv, h, w, c, generator=g).to(DEV)
    rows = ops.proj_rows(synthetic.synthetic_cameras(nv + 1, h * 4, w * 4, seed=3)["stage1"])[0]
    hyp = torch.linspace(425.0, 935.0, d).view(d, 1, 1).expand(d, h, w).contiguous()
    dsim = torch.randn(nv, d, h, w, generator=g).to(DEV)
    _, _, flag = ops.warp_corr_backward(ref, src, rows, hyp.to(DEV), dsim, planes=True)
    assert int(flag.item()) == 0
    hyp2 = hyp.clone()
    hyp2[3, 7, 9] += 1.0
    _, _, flag = ops.warp_corr_backward(ref, src, rows, hyp2.to(DEV), dsim, planes=True)
    assert int(flag.item()) & 2


def test_depth_stages_training_step():
    """A training step's three DepthNet stages (hypotheses, cost volume + its backward, view aggregation,
    train-mode PixelwiseNet and CostRegNets, softmax/WTA, trans_mvsnet_loss and d loss / d logits)
    against torch autograd through the oracle + oracle/loss_ref.py on the CPU (fp32), 128x160, N=3,
    8/8/8 hypotheses: loss value, d loss / d stage features, every CostRegNet and PixelwiseNet
    parameter gradient (1e-3 of each quantity's max magnitude), identical WTA depths."""
    import torch.nn.functional as F
    from oracle import loss_ref
    from transmvsnet_amd import TransMVSNet, synthetic
    from transmvsnet_amd.train import depth_stages_train
    H, W, N, ND = 128, 160, 3, (8, 8, 8)
    sd = golden_state_dict()
    model = TransMVSNet(ndepths=list(ND))
    model.load_state_dict(sd, strict=True)
    model = model.to(DEV)
    g = torch.Generator().manual_seed(9)
    feats = [{k: torch.randn(1, c, H // s, W // s, generator=g) for k, c, s in
              (("stage1", 32, 4), ("stage2", 16, 2), ("stage3", 8, 1))} for _ in range(N)]
    proj = synthetic.synthetic_cameras(N, H, W, seed=1)
    dv = synthetic.synthetic_depth_values(1)
    gt = {f"stage{s + 1}": 425.0 + 500.0 * torch.rand(1, H >> (2 - s), W >> (2 - s), generator=g) for s in range(3)}
    gt = {"stage1": gt["stage1"][:, :H // 4, :W // 4], "stage2": gt["stage2"][:, :H // 2, :W // 2], "stage3": gt["stage3"]}
    mask = {k: (torch.rand(v.shape, generator=g) > 0.3).float() for k, v in gt.items()}
    # GPU
    leaves = {k: torch.stack([f[k][0].permute(1, 2, 0) for f in feats]).contiguous().to(DEV).requires_grad_()
              for k in ("stage1", "stage2", "stage3")}
    total, outs = depth_stages_train(model, leaves, proj, dv.to(DEV), {k: v.to(DEV) for k, v in gt.items()},
                                     {k: v.to(DEV) for k, v in mask.items()}, (H, W))
    torch.cuda.synchronize()
    # CPU reference: the oracle in train mode, autograd
    rsd = {k: (v.clone().requires_grad_() if v.is_floating_point() and "running" not in k else v.clone())
           for k, v in sd.items()}
    rfe = [{k: v.clone().requires_grad_() for k, v in f.items()} for f in feats]
    outputs, depth, vw = {}, None, None
    for s in range(3):
        name = f"stage{s + 1}"
        hyp = oracle.stage_hypotheses(depth, dv, s, (H, W), ND)
        if s > 0:
            vw = F.interpolate(vw, scale_factor=2, mode="nearest")
        sim, vw_new = oracle.build_cost_volume(rsd, [f[name] for f in rfe], proj[name], hyp, vw if s else None,
                                               training=True)
        if s == 0:
            vw = vw_new.detach()
        logits = oracle.cost_reg_net(rsd, f"cost_regularization.{s}.", sim, training=True)[:, 0]
        prob = torch.exp(F.log_softmax(logits, dim=1))
        depth = torch.gather(hyp, 1, prob.argmax(1, keepdim=True)).squeeze(1)
        outputs[name] = {"prob_volume": prob, "depth_values": hyp}
        np.testing.assert_array_equal(outs[name]["depth_values"].cpu().numpy(), hyp.detach().numpy())
        assert torch.equal(outs[name]["depth"].cpu(), depth.clamp(425.0, 935.0).detach()), name
    ref_total = loss_ref.trans_mvsnet_loss(outputs, gt, mask, dlossw=(0.5, 1.0, 2.0))[0]
    ref_total.backward()
    rep = {"loss": abs(float(total) - float(ref_total)) / abs(float(ref_total))}
    assert rep["loss"] < 1e-5, rep
    worst = (0.0, None)
    for k in ("stage1", "stage2", "stage3"):
        for v in range(N):
            worst = max(worst, (_rel(leaves[k].grad[v].permute(2, 0, 1), rfe[v][k].grad[0]), f"d{k}[{v}]"))
    params = dict(model.named_parameters())
    for n, t in rsd.items():
        if t.requires_grad and (n.startswith("cost_regularization.") or n.startswith("DepthNet.")):
            assert params[n].grad is not None, n
            worst = max(worst, (_rel(params[n].grad, t.grad), n))
    rep["worst_grad"] = worst
    print(rep)
    assert worst[0] < 1e-3, rep


@pytest.mark.parametrize("stage", [1, 2])
def test_aggregate_and_pixelwise_train(stage):
    """View aggregation + (stage 1) train-mode PixelwiseNet on csrc/pw_train.hip against torch autograd
    through the oracle's pieces (pixelwise_net with batch statistics, the view-ordered weighted mean),
    C5 stage-1 size (48 x 144 x 192, 3 source views) / stage-2 size with given weights. The reference
    runs in fp32 and fp64: sim, view weights, d sims within 1e-4 of the fp32 reference; PixelwiseNet
    gradients within max(1e-4, 2 x the fp32 reference's own error) of fp64 (the BatchNorm backward
    sums cancel: conv0.conv.weight's gradient exists only through BatchNorm's eps, since BN removes
    the scale of a single-input 1x1 conv -- the fp32 reference gets it badly wrong, see the log)."""
    import torch.nn.functional as F
    from transmvsnet_amd import TransMVSNet
    from transmvsnet_amd.train import aggregate_train
    sd = golden_state_dict()
    model = TransMVSNet()
    model.load_state_dict(sd, strict=True)
    model = model.to(DEV)
    v, d, h, w = (3, 48, 144, 192) if stage == 1 else (3, 32, 288, 384)
    g = torch.Generator().manual_seed(31 + stage)
    sims = (torch.randn(v, d, h, w, generator=g) * 0.3).contiguous()
    dsim = torch.randn(d, h, w, generator=g)
    vw_small = torch.rand(v, h // 2, w // 2, generator=g) if stage == 2 else None
    sg = sims.to(DEV).requires_grad_()
    sim, vw = aggregate_train(sg, model, None if stage == 1 else vw_small.to(DEV), 0 if stage == 1 else 1)
    sim.backward(dsim.to(DEV))
    torch.cuda.synchronize()
    P = "DepthNet.pixel_wise_net."
    refs = {}
    for dt in (torch.float32, torch.float64):
        rsd = {k: (t.to(dt).clone().requires_grad_() if t.is_floating_point() and "running" not in k
                   else (t.to(dt).clone() if t.is_floating_point() else t.clone())) for k, t in sd.items()
               if k.startswith(P)}
        sc = sims.to(dt).clone().requires_grad_()
        sim_sum, w_sum, vws = 0, 1e-5, []
        for i in range(v):
            s_v = sc[i][None, None]
            if stage == 1:
                vw_i = oracle.pixelwise_net(rsd, s_v, training=True)[:, 0]
            else:
                vw_i = F.interpolate(vw_small.to(dt)[i][None, None], scale_factor=2, mode="nearest")[0]
            vws.append(vw_i)
            sim_sum = sim_sum + s_v[0] * vw_i.unsqueeze(1)
            w_sum = w_sum + vw_i.unsqueeze(1)
        ref = (sim_sum / w_sum)[0]
        ref.backward(dsim.to(dt))
        refs[dt] = (ref, sc.grad, torch.cat(vws, 0), rsd)
    ref, ref_ds, ref_vw, rsd = refs[torch.float32]
    ex, ex_ds, ex_vw, esd = refs[torch.float64]
    rep = {"sim": _rel(sim, ref), "dsims": _rel(sg.grad, ref_ds)}
    assert rep["sim"] < 1e-4 and rep["dsims"] < 1e-4, rep
    if stage == 1:
        rep["view_w"] = _rel(vw, ref_vw)
        assert rep["view_w"] < 1e-4, rep
        pw = model.DepthNet.pixel_wise_net
        grads = {"conv0.conv.weight": pw.conv0.conv.weight, "conv0.bn.weight": pw.conv0.bn.weight, "conv0.bn.bias": pw.conv0.bn.bias,
                 "conv1.conv.weight": pw.conv1.conv.weight, "conv1.bn.weight": pw.conv1.bn.weight,
                 "conv1.bn.bias": pw.conv1.bn.bias, "conv2.weight": pw.conv2.weight, "conv2.bias": pw.conv2.bias}
        for name, t in grads.items():
            e_gpu, e_ref = _rel(t.grad, esd[P + name].grad), _rel(rsd[P + name].grad, esd[P + name].grad)
            rep[name] = (e_gpu, e_ref)
            assert e_gpu <= max(1e-4, 2.0 * e_ref), (name, rep)
        for name, t in (("conv0.bn.running_mean", pw.conv0.bn.running_mean),
                        ("conv0.bn.running_var", pw.conv0.bn.running_var),
                        ("conv1.bn.running_mean", pw.conv1.bn.running_mean),
                        ("conv1.bn.running_var", pw.conv1.bn.running_var)):
            rep[name] = _rel(t, rsd[P + name])
            assert rep[name] < 1e-5, rep
    print(stage, rep)


def test_pathway_train_forward_backward():
    """FMT_with_pathway's lateral steps (models/FMT.py:201-209, 221-228) with their backward, C5 sizes
    (stage-1 FMT output 144x192x32, N=4 views), against torch autograd through the same ops on the CPU
    (fp32): stage-2/3 features, d FMT output, d FeatureNet stage-2/3 features, the four conv weight
    gradients -- 1e-4 of each quantity's max magnitude (the weight gradients sum ~1e5-1e6 terms)."""
    import torch.nn.functional as F
    from transmvsnet_amd import TransMVSNet
    from transmvsnet_amd.train import pathway_train
    sd = golden_state_dict()
    model = TransMVSNet()
    model.load_state_dict(sd, strict=True)
    model = model.to(DEV)
    n, h, w = 4, 144, 192
    g = torch.Generator().manual_seed(41)
    s1 = torch.randn(n, 32, h, w, generator=g)
    s2 = torch.randn(n, 16, 2 * h, 2 * w, generator=g)
    s3 = torch.randn(n, 8, 4 * h, 4 * w, generator=g)
    d2 = torch.randn(n, 16, 2 * h, 2 * w, generator=g)
    d3 = torch.randn(n, 8, 4 * h, 4 * w, generator=g)
    a1 = s1.permute(0, 2, 3, 1).contiguous().to(DEV).requires_grad_()
    a2, a3 = s2.to(DEV).requires_grad_(), s3.to(DEV).requires_grad_()
    o2, o3 = pathway_train(model, a1, a2, a3)
    torch.autograd.backward([o2, o3], [d2.permute(0, 2, 3, 1).contiguous().to(DEV),
                                       d3.permute(0, 2, 3, 1).contiguous().to(DEV)])
    torch.cuda.synchronize()
    P = "FMT_with_pathway."
    W = {k: sd[P + k].clone().requires_grad_() for k in ("dim_reduction_1.weight", "smooth_1.weight",
                                                         "dim_reduction_2.weight", "smooth_2.weight")}
    c1, c2, c3 = s1.clone().requires_grad_(), s2.clone().requires_grad_(), s3.clone().requires_grad_()
    r2 = F.conv2d(F.interpolate(F.conv2d(c1, W["dim_reduction_1.weight"]), size=(2 * h, 2 * w), mode="bilinear") + c2,
                  W["smooth_1.weight"], padding=1)
    r3 = F.conv2d(F.interpolate(F.conv2d(r2, W["dim_reduction_2.weight"]), size=(4 * h, 4 * w), mode="bilinear") + c3,
                  W["smooth_2.weight"], padding=1)
    torch.autograd.backward([r2, r3], [d2, d3])
    fp = model.FMT_with_pathway
    rep = {"stage2": _rel(o2.permute(0, 3, 1, 2), r2), "stage3": _rel(o3.permute(0, 3, 1, 2), r3),
           "d_fmt_out": _rel(a1.grad.permute(0, 3, 1, 2), c1.grad), "d_stage2": _rel(a2.grad, c2.grad),
           "d_stage3": _rel(a3.grad, c3.grad),
           "dim_reduction_1": _rel(fp.dim_reduction_1.weight.grad, W["dim_reduction_1.weight"].grad),
           "smooth_1": _rel(fp.smooth_1.weight.grad, W["smooth_1.weight"].grad),
           "dim_reduction_2": _rel(fp.dim_reduction_2.weight.grad, W["dim_reduction_2.weight"].grad),
           "smooth_2": _rel(fp.smooth_2.weight.grad, W["smooth_2.weight"].grad)}
    print(rep)
    assert all(v < 1e-4 for v in rep.values()), rep


@pytest.mark.parametrize("with_fmt,loss", [(False, "trans_mvsnet"), (True, "trans_mvsnet"), (True, "focal_bld")])
def test_training_step_from_fmt_output(with_fmt, loss):
    """The training step from the FMT output (with_fmt: from FeatureNet's stage-1 output, the FMT's 8
    encoder layers included) and FeatureNet's stage-2/3 features on: FMT_with_pathway's lateral steps,
    then the three DepthNet stages and trans_mvsnet_loss (all HIP), against torch autograd through the
    same chain on the CPU (128x160, N=3, 8/8/8): loss, d stage-1 input, d FeatureNet stage-2/3
    features, the pathway (and FMT) weight gradients (1e-3 of max magnitude). loss="focal_bld" is
    config C5's loss (finetune.py:159, focal_loss_bld with dlossw 1,1,1) and also checks its EPE /
    less1 / less3 against the reference's."""
    import torch.nn.functional as F
    from oracle import loss_ref
    from transmvsnet_amd import TransMVSNet, synthetic
    from transmvsnet_amd.train import depth_stages_train, fmt_train, pathway_train
    H, W, N, ND = 128, 160, 3, (8, 8, 8)
    sd = golden_state_dict()
    model = TransMVSNet(ndepths=list(ND))
    model.load_state_dict(sd, strict=True)
    model = model.to(DEV)
    g = torch.Generator().manual_seed(19)
    s1 = torch.randn(N, 32, H // 4, W // 4, generator=g)
    s2 = torch.randn(N, 16, H // 2, W // 2, generator=g)
    s3 = torch.randn(N, 8, H, W, generator=g)
    proj = synthetic.synthetic_cameras(N, H, W, seed=1)
    dv = synthetic.synthetic_depth_values(1)
    gt = {f"stage{s + 1}": 425.0 + 500.0 * torch.rand(1, H >> (2 - s), W >> (2 - s), generator=g) for s in range(3)}
    mask = {k: (torch.rand(v.shape, generator=g) > 0.3).float() for k, v in gt.items()}
    a1 = (s1 if with_fmt else s1.permute(0, 2, 3, 1)).contiguous().to(DEV).requires_grad_()
    a2, a3 = s2.to(DEV).requires_grad_(), s3.to(DEV).requires_grad_()
    st1 = fmt_train(model, a1) if with_fmt else a1
    st2, st3 = pathway_train(model, st1, a2, a3)
    dlossw = (1.0, 1.0, 1.0) if loss == "focal_bld" else (0.5, 1.0, 2.0)
    dint = float(dv[0, 1] - dv[0, 0])
    total, outs = depth_stages_train(model, {"stage1": st1, "stage2": st2, "stage3": st3}, proj, dv.to(DEV),
                                     {k: v.to(DEV) for k, v in gt.items()}, {k: v.to(DEV) for k, v in mask.items()},
                                     (H, W), dlossw=dlossw, loss=loss, depth_interval=dint)
    torch.cuda.synchronize()
    P = "FMT_with_pathway."
    metrics = {}

    def reference(dt):
        rsd = {k: (v.to(dt).clone().requires_grad_() if v.is_floating_point() and "running" not in k
                   else (v.to(dt).clone() if v.is_floating_point() else v.clone())) for k, v in sd.items()}
        c1, c2, c3 = (x.to(dt).clone().requires_grad_() for x in (s1, s2, s3))
        f1 = c1
        if with_fmt:
            ref_list = oracle.fmt_ref(rsd, c1[:1])
            f1 = torch.cat([ref_list[-1]] + [oracle.fmt_src(rsd, ref_list, c1[i:i + 1]) for i in range(1, N)])
        r2 = F.conv2d(F.interpolate(F.conv2d(f1, rsd[P + "dim_reduction_1.weight"]), size=(H // 2, W // 2),
                                    mode="bilinear") + c2, rsd[P + "smooth_1.weight"], padding=1)
        r3 = F.conv2d(F.interpolate(F.conv2d(r2, rsd[P + "dim_reduction_2.weight"]), size=(H, W), mode="bilinear")
                      + c3, rsd[P + "smooth_2.weight"], padding=1)
        feats = {"stage1": f1, "stage2": r2, "stage3": r3}
        outputs, depth, vw = {}, None, None
        for s in range(3):
            name = f"stage{s + 1}"
            hyp = oracle.stage_hypotheses(depth, dv.to(dt), s, (H, W), ND)
            if s > 0:
                vw = F.interpolate(vw, scale_factor=2, mode="nearest")
            sim, vw_new = oracle.build_cost_volume(rsd, [feats[name][i:i + 1] for i in range(N)], proj[name].to(dt),
                                                   hyp, vw if s else None, training=True)
            if s == 0:
                vw = vw_new.detach()
            logits = oracle.cost_reg_net(rsd, f"cost_regularization.{s}.", sim, training=True)[:, 0]
            prob = torch.exp(F.log_softmax(logits, dim=1))
            depth = torch.gather(hyp, 1, prob.argmax(1, keepdim=True)).squeeze(1)
            outputs[name] = {"prob_volume": prob, "depth_values": hyp, "depth": depth.clamp(425.0, 935.0)}
        gtd, mkd = {k: v.to(dt) for k, v in gt.items()}, {k: v.to(dt) for k, v in mask.items()}
        if loss == "focal_bld":
            res = loss_ref.focal_loss_bld(outputs, gtd, mkd, dint, dlossw=dlossw)
            metrics[dt] = [float(x) for x in res[1:]]
        else:
            res = loss_ref.trans_mvsnet_loss(outputs, gtd, mkd, dlossw=dlossw)
        tot = res[0]
        tot.backward()
        grads = {"d_stage1_input": c1.grad, "d_stage2": c2.grad, "d_stage3": c3.grad}
        grads.update({n: rsd[n].grad for n in sd if n.startswith(P) and rsd[n].grad is not None})
        return float(tot), grads

    params = dict(model.named_parameters())
    got = {"d_stage1_input": a1.grad if with_fmt else a1.grad.permute(0, 3, 1, 2), "d_stage2": a2.grad,
           "d_stage3": a3.grad}
    ref_total, r32 = reference(torch.float32)
    names = ["d_stage1_input", "d_stage2", "d_stage3"] + [P + k for k in ("dim_reduction_1.weight", "smooth_1.weight",
                                                                          "dim_reduction_2.weight", "smooth_2.weight")]
    if with_fmt:
        names += [n for n in r32 if ".FMT." in n]
    got.update({n: params[n].grad for n in names if n.startswith(P)})
    rep = {"loss": abs(float(total) - ref_total) / abs(ref_total)}
    assert rep["loss"] < 1e-5, rep
    if loss == "focal_bld":  # depth_loss, epe, less1, less3 of the stage-3 WTA depth
        got_m = [float(outs["metrics"][k]) for k in ("depth_loss", "epe", "less1", "less3")]
        # (a near-tie WTA flip moves one pixel of 20,480: rtol 1e-3)
        assert np.allclose(got_m, metrics[torch.float32], rtol=1e-3, atol=1e-4), (got_m, metrics[torch.float32])
    if not with_fmt:
        rep.update({n: _rel(got[n], r32[n]) for n in names})
        print(rep)
        assert all(v < 1e-3 for v in rep.values()), rep
        return
    # with the FMT in the chain the fp32 reference's own gradients drift 1e-3..1e-2 from exact: judge vs fp64
    _, r64 = reference(torch.float64)
    errs = {n: (_rel(got[n], r64[n]), _rel(r32[n], r64[n])) for n in names}
    ref_worst = max(e for _, e in errs.values())
    print(rep, {n: (f"{a:.1e}", f"{b:.1e}") for n, (a, b) in errs.items() if ".FMT." not in n},
          "FMT worst (gpu, fp32 ref):", max(errs[n] for n in names if ".FMT." in n), "fp32 ref worst:", ref_worst)
    for n, (e_gpu, e_ref) in errs.items():
        assert e_gpu <= max(1e-3, 2.0 * e_ref, ref_worst), (n, e_gpu, e_ref, ref_worst)


def _fmt_ref_sd(sd, dt):
    return {k: v.to(dt).clone().requires_grad_() for k, v in sd.items() if k.startswith("FMT_with_pathway.FMT.")}


@pytest.mark.parametrize("self_attn,L", [(True, 320), (False, 320), (True, 27648), (False, 27648)])
def test_encoder_layer_backward(self_attn, L):
    """One EncoderLayer's backward on the HIP token kernels (models/FMT.py:96-111; 3 views x 320
    tokens; a cross layer's queries are the 2 source views, its K/V the reference tokens) against
    torch autograd through oracle.encoder_layer in fp64: dx, d source, all 16 parameter gradients
    within max(1e-4, 2 x the fp32 reference's own error) of each quantity's max magnitude."""
    from transmvsnet_amd.train import _ENC_PARAMS, _encoder_layer_backward, _pack_enc
    sd = golden_state_dict()
    i = 0 if self_attn else 1
    P = f"FMT_with_pathway.FMT.layers.{i}."
    g = torch.Generator().manual_seed(5 + i)
    nv = 3
    x = torch.randn(nv, L, 32, generator=g)
    dy = torch.randn(nv, L, 32, generator=g)
    refs = {}
    for dt in (torch.float32, torch.float64):
        rsd = _fmt_ref_sd(sd, dt)
        xc = x.to(dt).clone().requires_grad_()
        if self_attn:
            out = oracle.encoder_layer(rsd, P, xc, xc)
            out.backward(dy.to(dt))
            refs[dt] = (out, xc.grad, None, rsd)
        else:
            out = oracle.encoder_layer(rsd, P, xc[1:], xc[:1].expand(nv - 1, L, 32))
            out.backward(dy[1:].to(dt))
            refs[dt] = (out, xc.grad[1:], xc.grad[0], rsd)
    p = [sd[P + n].to(DEV).contiguous() for n in _ENC_PARAMS]
    xd = x.to(DEV)
    if self_attn:
        dx, dsrc, grads = _encoder_layer_backward(p, _pack_enc(p), xd.view(-1, 32), xd.view(-1, 32),
                                                  dy.to(DEV).view(-1, 32), L, L, True)
    else:
        dx, dsrc, grads = _encoder_layer_backward(p, _pack_enc(p), xd[1:].reshape(-1, 32), xd[0].contiguous(),
                                                  dy[1:].to(DEV).reshape(-1, 32), (nv - 1) * L, L, False)
    torch.cuda.synchronize()
    (_, r_dx, r_ds, rsd32), (_, e_dx, e_ds, rsd64) = refs[torch.float32], refs[torch.float64]
    checks = [("dx", dx.view_as(e_dx), r_dx, e_dx)]
    if not self_attn:
        checks.append(("dsrc", dsrc.view_as(e_ds), r_ds, e_ds))
    checks += [(n, gr, rsd32[P + n].grad, rsd64[P + n].grad) for n, gr in zip(_ENC_PARAMS, grads)]
    errs = [(n, _rel(got.reshape(r64.shape), r64), _rel(r32, r64)) for n, got, r32, r64 in checks]
    print("self" if self_attn else "cross", L, [(n, f"{a:.1e}", f"{b:.1e}") for n, a, b in errs])
    for n, e_gpu, e_ref in errs:
        assert e_gpu <= max(1e-4, 2.0 * e_ref), (n, e_gpu, e_ref)


@pytest.mark.parametrize("nv,h,w", [(3, 16, 20), (4, 144, 192)])
def test_fmt_train_forward_backward(nv, h, w):
    """The whole FMT for training (models/FMT.py:147-177: 4 self + 4 cross layers, reference view first)
    at a small shape and the C5 stage-1 shape (BlendedMVS 768x576 -> 144x192, N=4): HIP forward against
    the fp32 oracle (1e-4 of max magnitude), d stage-1 features and all 128 parameter gradients against
    fp64 torch autograd through the oracle, within max(1e-4, 2 x the fp32 reference's own error, the
    fp32 reference's worst error over all gradients) of each quantity's max magnitude."""
    from transmvsnet_amd import TransMVSNet
    from transmvsnet_amd.train import _ENC_PARAMS, fmt_params, fmt_train
    sd = golden_state_dict()
    model = TransMVSNet()
    model.load_state_dict(sd, strict=True)
    model = model.to(DEV)
    g = torch.Generator().manual_seed(nv + h)
    s1 = torch.randn(nv, 32, h, w, generator=g)
    gout = torch.randn(nv, 32, h, w, generator=g)
    a1 = s1.to(DEV).requires_grad_()
    out = fmt_train(model, a1)
    out.backward(gout.permute(0, 2, 3, 1).contiguous().to(DEV))
    torch.cuda.synchronize()
    refs = {}
    for dt in (torch.float32, torch.float64):
        rsd = _fmt_ref_sd(sd, dt)
        xc = s1.to(dt).clone().requires_grad_()
        ref_list = oracle.fmt_ref(rsd, xc[:1])
        r = torch.cat([ref_list[-1]] + [oracle.fmt_src(rsd, ref_list, xc[i:i + 1]) for i in range(1, nv)])
        r.backward(gout.to(dt))
        refs[dt] = (r, xc.grad, rsd)
    (r32, dx32, rsd32), (_, dx64, rsd64) = refs[torch.float32], refs[torch.float64]
    fwd = _rel(out.permute(0, 3, 1, 2), r32)
    assert fwd < 1e-4, fwd
    names = [f"FMT_with_pathway.FMT.layers.{i}.{n}" for i in range(8) for n in _ENC_PARAMS]
    checks = [("d_stage1", a1.grad, dx32, dx64)] + [(n, p.grad, rsd32[n].grad, rsd64[n].grad)
                                                    for n, p in zip(names, fmt_params(model))]
    errs = [(n, _rel(got, e64), _rel(e32, e64)) for n, got, e32, e64 in checks]
    ref_worst = max(e for _, _, e in errs)
    worst = max((a, n, b) for n, a, b in errs)
    print((nv, h, w), {"forward": fwd, "d_stage1 (gpu, fp32 ref)": errs[0][1:], "worst (gpu, name, fp32 ref)": worst,
                       "fp32 ref worst": ref_worst})
    for n, e_gpu, e_ref in errs:
        assert e_gpu <= max(1e-4, 2.0 * e_ref, ref_worst), (n, e_gpu, e_ref, ref_worst)


def test_flat_adam_matches_torch_adam():
    """FlatAdam / tmvs_adam_step (finetune.py:324's optimizer: Adam, betas 0.9/0.999, eps 1e-8,
    weight_decay 1e-4, lr 1e-3) against torch.optim.Adam (single-tensor, CPU fp32) over 5 steps on
    the CostRegNet parameters with random gradients: parameters and both moments within 2e-6 of
    each quantity's max magnitude (fma contraction vs torch's separate ops: ulp-level)."""
    from transmvsnet_amd.train import FlatAdam
    sd = {k[len("cost_regularization.0."):]: v for k, v in golden_state_dict().items()
          if k.startswith("cost_regularization.0.")}
    cr_gpu, cr_cpu = CostRegNet(1, 8), CostRegNet(1, 8)
    cr_gpu.load_state_dict(sd, strict=True)
    cr_cpu.load_state_dict(sd, strict=True)
    cr_gpu = cr_gpu.to(DEV)
    pg = [p for p in cr_gpu.parameters()]
    pc = [p for p in cr_cpu.parameters()]
    opt = FlatAdam(pg, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4)
    ref = torch.optim.Adam(pc, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-4, foreach=False)
    g = torch.Generator().manual_seed(3)
    for _ in range(5):
        grads = [torch.randn(p.shape, generator=g) * 0.1 for p in pc]
        opt.zero_grad()
        ref.zero_grad()
        for p, q, gr in zip(pg, pc, grads):
            p.grad = gr.to(DEV)
            q.grad = gr.clone()
        opt.step()
        ref.step()
    torch.cuda.synchronize()
    worst = 0.0
    off = 0
    for p, q in zip(pg, pc):
        st = ref.state[q]
        n = q.numel()
        for got, exp in ((p, q), (opt.exp_avg[off:off + n].view_as(q), st["exp_avg"]),
                         (opt.exp_avg_sq[off:off + n].view_as(q), st["exp_avg_sq"])):
            worst = max(worst, _rel(got, exp))
        off += n
    print("FlatAdam vs torch.optim.Adam, worst relative difference:", worst)
    assert worst < 2e-6, worst


def test_flat_adam_graph_replay_equals_eager_steps():
    """A FlatAdam step captured in a HIP graph (tmvs_adam_step_dev: the step number advanced on the
    device per replay) gives bitwise the same parameters and moments as eager steps (host step
    number), after 2 eager steps and 3 replays vs 5 eager steps with the same gradients; and an
    eager step after the replays is step 6 (the capture does not count as a step, the replays do)."""
    from transmvsnet_amd.train import FlatAdam
    torch.manual_seed(5)
    shapes = [(8, 1, 3, 3, 3), (16,), (64, 32)]
    init = [torch.randn(s) for s in shapes]
    grads = [torch.randn(s).to(DEV) * 0.1 for s in shapes]
    pa = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    pb = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    oa = FlatAdam(pa, lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4)
    ob = FlatAdam(pb, lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4)
    for _ in range(5):
        oa.zero_grad()
        for p, gr in zip(pa, grads):
            p.grad = gr.clone()
        oa.step()

    def step_b():
        ob.zero_grad()
        for p, gr in zip(pb, grads):
            p.grad = gr.clone()
        ob.step()
    for _ in range(2):
        step_b()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step_b()  # captured: its launches run only on replay
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    assert int(ob._step_dev.item()) == 5 and ob.step_count == 5
    assert torch.equal(oa.flat, ob.flat)
    assert torch.equal(oa.exp_avg, ob.exp_avg) and torch.equal(oa.exp_avg_sq, ob.exp_avg_sq)
    oa.zero_grad()
    for p, gr in zip(pa, grads):
        p.grad = gr.clone()
    oa.step()
    step_b()  # eager, after the capture
    torch.cuda.synchronize()
    assert oa.step_count == 6 and ob.step_count == 6
    assert torch.equal(oa.flat, ob.flat)
    assert torch.equal(oa.exp_avg, ob.exp_avg) and torch.equal(oa.exp_avg_sq, ob.exp_avg_sq)


def test_flat_adam_graph_replay_follows_lr_schedule():
    """A captured FlatAdam step reads its learning rate from the device when the replay runs (ABI 8,
    ADVICE r4): replays with opt.lr changed before each (sync_lr) give bitwise the parameters and
    moments of eager steps run with the same per-step learning rates (finetune.py:58-72's
    WarmupMultiStepLR sets the lr every iteration)."""
    from transmvsnet_amd.train import FlatAdam
    torch.manual_seed(6)
    shapes = [(8, 4, 3, 3, 3), (32,)]
    init = [torch.randn(s) for s in shapes]
    grads = [torch.randn(s).to(DEV) * 0.1 for s in shapes]
    lrs = [1e-3, 1e-3, 5e-4, 1e-4, 2e-3]
    pa = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    pb = [torch.nn.Parameter(t.clone().to(DEV)) for t in init]
    oa = FlatAdam(pa, lr=1e-3, weight_decay=1e-4)
    ob = FlatAdam(pb, lr=1e-3, weight_decay=1e-4)
    for lr in lrs:
        oa.zero_grad()
        for p, gr in zip(pa, grads):
            p.grad = gr.clone()
        oa.step(lr=lr)

    def step_b():
        ob.zero_grad()
        for p, gr in zip(pb, grads):
            p.grad = gr.clone()
        ob.step()
    step_b()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step_b()
    for lr in lrs[1:]:
        ob.lr = lr
        ob.sync_lr()
        graph.replay()
    torch.cuda.synchronize()
    assert ob.step_count == len(lrs)
    assert torch.equal(oa.flat, ob.flat)
    assert torch.equal(oa.exp_avg, ob.exp_avg) and torch.equal(oa.exp_avg_sq, ob.exp_avg_sq)


def test_graph_overflow_flags_are_sticky():
    """The overflow flag of a warp backward captured in a HIP graph is sticky: a replay
    whose d similarity is non-finite followed by a clean replay still raises at the next check; the
    check clears the flags, so a clean replay afterwards passes."""
    from transmvsnet_amd import ops, synthetic
    from transmvsnet_amd import train as tr
    c, d, h, w, nv = 8, 8, 24, 32, 2
    g = torch.Generator().manual_seed(7)
    ref = torch.randn(h, w, c, generator=g).to(DEV).requires_grad_()
    src = torch.randn(nv, h, w, c, generator=g).to(DEV).requires_grad_()
    rows = ops.proj_rows(synthetic.synthetic_cameras(nv + 1, h * 4, w * 4, seed=3)["stage1"])[0]
    hyp = torch.linspace(425.0, 935.0, d).view(d, 1, 1).expand(d, h, w).contiguous().to(DEV)
    clean = torch.randn(nv, d, h, w, generator=g).to(DEV)
    dsim = clean.clone()
    tr.warp_corr_views(ref, src, hyp, rows).backward(dsim)  # eager: reserves the flag arena
    tr.drop_graph_flags()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        tr.warp_corr_views(ref, src, hyp, rows).backward(dsim)
    assert len(tr.GRAPH_FLAGS) == 1
    try:
        graph.replay()
        tr.check_graph_flags()  # clean
        dsim[0, 3, 5, 7] = float("inf")
        graph.replay()  # overflows
        dsim.copy_(clean)
        graph.replay()  # clean again: the earlier overflow must not be lost
        with pytest.raises(RuntimeError, match="non-finite"):
            tr.check_graph_flags()
        graph.replay()
        tr.check_graph_flags()  # cleared by the previous check
    finally:
        tr.drop_graph_flags()


def test_training_loop_reduces_loss():
    """A C5-style loop on one fixed synthetic sample (128x160, N=3, 8/8/8): FMT -> pathway -> DepthNet
    stages -> focal_loss_bld (dlossw 1,1,1) -> backward -> FlatAdam.step, 8 iterations, all HIP. The
    loss must fall (the optimizer and every backward kernel point downhill together), stay finite,
    and the BatchNorm running statistics must move."""
    from transmvsnet_amd import TransMVSNet, synthetic
    from transmvsnet_amd.train import FlatAdam, depth_stages_train, fmt_train, pathway_train
    H, W, N, ND = 128, 160, 3, (8, 8, 8)
    model = TransMVSNet(ndepths=list(ND))
    model.load_state_dict(golden_state_dict(), strict=True)
    model = model.to(DEV)
    g = torch.Generator().manual_seed(23)
    feats = [torch.randn(N, c, H // s, W // s, generator=g).to(DEV) for c, s in ((32, 4), (16, 2), (8, 1))]
    proj = synthetic.synthetic_cameras(N, H, W, seed=1)
    dv = synthetic.synthetic_depth_values(1).to(DEV)
    gt = {f"stage{s + 1}": (425.0 + 500.0 * torch.rand(1, H >> (2 - s), W >> (2 - s), generator=g)).to(DEV)
          for s in range(3)}
    mask = {k: torch.ones_like(v) for k, v in gt.items()}
    params = [p for n, p in model.named_parameters()
              if n.startswith(("cost_regularization.", "DepthNet.", "FMT_with_pathway."))]
    opt = FlatAdam(params, lr=1e-3, weight_decay=1e-4)
    rm0 = model.cost_regularization[0].conv0.bn.running_mean.clone()
    losses = []
    for _ in range(8):
        opt.zero_grad()
        st1 = fmt_train(model, feats[0])
        st2, st3 = pathway_train(model, st1, feats[1], feats[2])
        total, _ = depth_stages_train(model, {"stage1": st1, "stage2": st2, "stage3": st3}, proj, dv, gt, mask,
                                      (H, W), dlossw=(1.0, 1.0, 1.0), loss="focal_bld",
                                      depth_interval=float(dv[0, 1] - dv[0, 0]))
        opt.allreduce()
        opt.step()
        losses.append(float(total))
    print("losses:", [f"{x:.4f}" for x in losses])
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < 0.9 * losses[0], losses
    assert not torch.equal(model.cost_regularization[0].conv0.bn.running_mean, rm0)


def test_bn_grouped_matches_per_group():
    """tmvs_bn_*_grouped (FeatureNet's per-view BatchNorm2d in one launch per pass) against torch
    autograd of relu(batch_norm(training=True)) applied to each group separately, with the parameter
    gradients summed over the groups. Bar: 1e-5 of each quantity's max |value|."""
    import torch.nn.functional as F
    from transmvsnet_amd import ops
    torch.manual_seed(3)
    g, h, w, c = 4, 23, 37, 16
    z = torch.randn(g, h, w, c) * 2 + 0.3
    dy = torch.randn(g, h, w, c)
    gamma = torch.rand(c) + 0.5
    beta = torch.randn(c) * 0.2
    gm, gb = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    zr = z.clone().requires_grad_()
    ys = []
    for v in range(g):
        x = zr[v].permute(2, 0, 1).unsqueeze(0)
        ys.append(F.relu(F.batch_norm(x, None, None, gm, gb, True, 0.1, 1e-5))[0].permute(1, 2, 0))
    y = torch.stack(ys)
    (y * dy).sum().backward()
    zd = z.to(DEV)
    mean, var = ops.bn_stats_grouped(zd)
    yd = ops.bn_relu_train_grouped(zd, mean, var, gamma.to(DEV), beta.to(DEV), 1e-5)
    dz, dg, db = ops.bn_relu_backward_grouped(dy.to(DEV), zd, mean, var, gamma.to(DEV), beta.to(DEV), 1e-5)
    for v in range(g):
        assert _rel(mean[v], z[v].reshape(-1, c).mean(0)) < 1e-6
        assert _rel(var[v], z[v].reshape(-1, c).var(0, unbiased=False)) < 1e-5
    for got, ref, tag in ((yd, y, "y"), (dz, zr.grad, "dz"), (dg, gm.grad, "dgamma"), (db, gb.grad, "dbeta")):
        assert _rel(got, ref) < 1e-5, tag
