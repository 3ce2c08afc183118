"""Training path: the differentiable blocks that run on HIP.

* ``fmt_train``: the FMT (models/FMT.py:96-177, 8 EncoderLayers) with its backward on the token
  kernels of csrc/fmt_train.hip (``_encoder_layer_backward``); ``pathway_train``: FMT_with_pathway's
  lateral steps (FMT.py:201-228) with their backward (csrc/pathway_train.hip + the generic convs).
* ``warp_corr_views``: the per-view similarity volumes of DepthNet (homo_warping + (warped *
  ref).mean(1), models/module.py:284-322, TransMVSNet.py:80) with the backward into the reference
  and source features (tmvs_warp_corr_backward: gather for the reference, deterministic
  fixed-point scatter for the sources, flushed wave-cooperatively).
* ``costregnet_train``: CostRegNet in train mode with its backward on csrc/costreg_train.hip.
* ``depth_stages_train``: the three DepthNet stages of a training step (models/TransMVSNet.py:38-109,
  174-221) from the FMT/pathway features to trans_mvsnet_loss (module.py:534-558) and its backward:
  hypotheses (tmvs_stage_hypotheses), per-view cost volumes (above), the view aggregation and the
  stage-1 PixelwiseNet in train mode (``aggregate_train``: csrc/pw_train.hip), CostRegNet (above),
  softmax/WTA (tmvs_softmax_wta) and the loss with d loss / d logits (tmvs_entropy_loss); gradients
  reach the stage features, the CostRegNet and PixelwiseNet parameters. Torch only packs
  parameters and sums gradients that meet.

``costregnet_train(module, x)`` is CostRegNet.forward (models/module.py:447-456) of a
``transmvsnet_amd.model.CostRegNet`` whose BatchNorm3d layers run in train mode, as in the
reference's training loop (train.py:137-161 / finetune.py:144-195, ``model.train()``):

  * forward: per layer tmvs_conv3d_generic (no bias) -> tmvs_bn_stats (batch mean, biased
    variance) -> tmvs_bn_relu_train (+ the U-Net skip); prob is a plain conv; the module's
    running_mean / running_var (unbiased) / num_batches_tracked are updated as nn.BatchNorm3d
    updates them (momentum 0.1);
  * backward (torch.autograd.Function): tmvs_bn_relu_backward per layer, the data gradient by
    tmvs_conv3d_generic with the gather transposed (Conv3d) or strided (ConvTranspose3d), gradients
    meeting at a skip accumulated in place (TMVS_CONV_ACCUMULATE), weight gradients by
    tmvs_conv3d_wgrad.

Input x [B, D, H, W] (the aggregated similarity volume; D, H, W divisible by 8), output the logits
[B, D, H, W]; d loss / d logits comes from transmvsnet_amd.loss (return_grad=True) or from torch.
Gradients flow to x (toward the cost volume) and to every conv weight and BN affine parameter.
Tensor layout is NDHWC throughout; weight re-layouts are index permutations (packs below).
"""
from __future__ import annotations

import torch

from . import ops
from .bn_running import update_running_stats
from .packing import gather_packs

# (name, stride, transposed, skip source) in forward order; channels from the module
_LAYERS = (("conv0", 1, False, None), ("conv1", 2, False, None), ("conv2", 1, False, None),
           ("conv3", 2, False, None), ("conv4", 1, False, None), ("conv5", 2, False, None),
           ("conv6", 1, False, None), ("conv7", 2, True, "conv4"), ("conv9", 2, True, "conv2"),
           ("conv11", 2, True, "conv0"))
BN_MOMENTUM = 0.1


class _WarpCorrViews(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ref, src, hyp, proj12, rot_order, planes):
        v, h, w, c = src.shape
        d = hyp.shape[0]
        sims = torch.empty(v, d, h, w, device=src.device)
        ones = torch.ones(1, 1, h, w, device=src.device)
        wsum = torch.empty(1, h, w, device=src.device)
        for i in range(v):  # one view per launch, weight 1, partial: sim_out = 1 * sim_v exactly
            ops.warp_corr(ref[None], src[i:i + 1][None], proj12[None, i:i + 1], hyp[None], view_w_in=ones, vw_shift=0,
                          vw_total=1, partial=True, sim_out=sims[i:i + 1], wsum_out=wsum, rot_order=rot_order)
        ctx.save_for_backward(ref, src, hyp)
        ctx.proj12, ctx.rot_order, ctx.planes = proj12, rot_order, planes
        return sims

    @staticmethod
    def backward(ctx, dsims):
        ref, src, hyp = ctx.saved_tensors
        if not torch.cuda.is_current_stream_capturing():
            reserve_graph_flags(ref.device, 8)
        dref, dsrc, flag = ops.warp_corr_backward(ref, src, ctx.proj12, hyp, dsims.contiguous(), ctx.rot_order,
                                                  planes=ctx.planes)
        if _DEFERRED_FLAGS is not None:  # inside depth_stages_train: one host sync after the whole backward
            _DEFERRED_FLAGS.append(flag.clone())
        elif torch.cuda.is_current_stream_capturing():  # a HIP-graph capture: checked after the replays
            GRAPH_FLAGS.append(_sticky_flag(flag))
        else:
            _check_overflow([flag])
        return dref, dsrc, None, None, None, None


_DEFERRED_FLAGS = None
# Sticky overflow flags of warp backwards captured in a HIP graph: one int32 per captured backward,
# OR-ed with that backward's flag word on every replay (the warp kernel clears its own flag word per
# launch, so a plain copy would keep only the last replay's). They live in a zeroed arena allocated
# outside any capture (a fill recorded inside the graph would clear them per replay).
GRAPH_FLAGS = []
_FLAG_ARENA = {}  # device index -> [arena int32 tensor, next free slot]
_ARENA_SLOTS = 256


def reserve_graph_flags(device, n=64):
    """Make sure >= n sticky-flag slots are free on `device` (call outside a capture; TrainStepGraph
    does). Eager warp backwards reserve them too, so a capture after an eager step finds them."""
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("reserve_graph_flags: call outside a HIP-graph capture")
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    a = _FLAG_ARENA.get(idx)
    if a is None or a[0].numel() - a[1] < n:
        _FLAG_ARENA[idx] = [torch.zeros(max(_ARENA_SLOTS, n), dtype=torch.int32, device=f"cuda:{idx}"), 0]


def _sticky_flag(flag):
    """Inside a capture: a zeroed arena slot that the graph ORs `flag` into on every replay."""
    idx = flag.device.index
    a = _FLAG_ARENA.get(idx)
    if a is None or a[1] >= a[0].numel():
        raise RuntimeError("warp_corr_backward captured in a HIP graph with no free overflow-flag slot: run one "
                           "eager step (or train.reserve_graph_flags(device)) before the capture")
    s = a[0][a[1]:a[1] + 1]
    a[1] += 1
    s.bitwise_or_(flag.reshape(1))
    return s


def check_graph_flags():
    """The overflow check of the warp backwards captured outside a TrainStepGraph (one host sync):
    raises if any of their replays since the last check overflowed. The flags stay registered (later
    replays are checked by later calls) and are cleared after each check; `drop_graph_flags` forgets
    them once their graph is gone."""
    try:
        _check_overflow(GRAPH_FLAGS)
    finally:
        for f in GRAPH_FLAGS:
            f.zero_()


def drop_graph_flags():
    GRAPH_FLAGS.clear()


def _check_overflow(flags):
    if not flags:
        return
    bits = int(torch.stack([f.reshape(()) for f in flags]).max().item())  # flag words are 0 when clean
    if bits:
        raise RuntimeError("warp_corr_backward: non-finite d similarity or reference features (bit 1: the "
                           "fixed-point scatter needs finite values) or non-planar hypotheses under planes=True "
                           f"(bit 2); flag {bits}")


def warp_corr_views(ref_nhwc, src_nhwc, hyp, proj12, rot_order="auto", planes=False):
    """Per-view similarity volumes sim_v [V, D, H, W] for ONE sample (ref [H,W,C], src [V,H,W,C] NHWC,
    hyp [D,H,W], proj12 HOST [V,12] from ops.proj_rows), differentiable w.r.t. ref and src. planes:
    hyp[d] holds one depth per plane (stage 1), so the backward gathers d src (TMVS_WARP_BWD_PLANES)."""
    if not src_nhwc.is_cuda:
        raise RuntimeError("warp_corr_views runs on the GPU only (no CPU fallback)")
    return _WarpCorrViews.apply(ref_nhwc.contiguous(), src_nhwc.contiguous(), hyp.contiguous(), proj12, rot_order,
                                planes)


class _PathwayStep(torch.autograd.Function):
    """One FMT_with_pathway lateral step (models/FMT.py:201-209, 221-228) with its backward:
    out = smooth(up2(reduce(coarse)) + lateral). coarse [N,h,w,cc] NHWC, lateral [N,cf,2h,2w] NCHW ->
    out [N,2h,2w,cf] NHWC. Forward: the fused inference kernel (tmvs_fmt_pathway); backward on the 2-D
    training convs of FeatureNet: the smoothing's data gradient as a forward conv of the flipped,
    transposed weight on the MFMA kernels (featurenet_train.dgrad_same), its weight gradient
    (tmvs_conv2d_wgrad), the interpolation's adjoint (tmvs_upsample2_backward_nhwc), the 1x1
    reduction's gradients (tmvs_conv2d_generic / tmvs_conv2d_wgrad)."""

    @staticmethod
    def forward(ctx, coarse, lateral, w_reduce, w_smooth):
        cf, cc = w_reduce.shape[0], w_reduce.shape[1]
        wr = w_reduce.detach().float().reshape(cf, cc).t().contiguous()
        ws = w_smooth.detach().float().permute(1, 2, 3, 0).contiguous()
        out = ops.fmt_pathway(coarse.contiguous(), lateral.contiguous(), wr, ws)
        ctx.save_for_backward(coarse, lateral, w_reduce, w_smooth)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .featurenet_train import _taps, _taps_t, _untaps, dgrad_same
        coarse, lateral, w_reduce, w_smooth = ctx.saved_tensors
        n, h, w, cc = coarse.shape
        cf = w_reduce.shape[0]
        dout = dout.contiguous()
        coarse = coarse.contiguous()
        # recompute u = up2(reduce(coarse)) + lateral (the fused forward keeps no intermediate)
        r = ops.conv2d_generic(coarse, _taps(w_reduce), cf, (h, w), 1, 1, 0)
        u = ops.upsample2_add_nhwc(r, lateral.contiguous())
        du = dgrad_same(dout, w_smooth, (2 * h, 2 * w))
        dws = _untaps(ops.conv2d_wgrad(dout, u.view(n, 2 * h, 2 * w, cf), 3, 1, 1), w_smooth.shape)
        dlat = du.permute(0, 3, 1, 2).contiguous()
        dr = ops.upsample2_backward_nhwc(du)
        dcoarse = ops.conv2d_generic(dr, _taps_t(w_reduce), cc, (h, w), 1, 1, 0)
        dwr = _untaps(ops.conv2d_wgrad(dr, coarse, 1, 1, 0), w_reduce.shape)
        return dcoarse, dlat, dwr, dws


def pathway_train(model, stage1_nhwc, stage2_nchw, stage3_nchw):
    """FMT_with_pathway's stage-2/3 features (models/FMT.py:221-228) from the FMT output stage1_nhwc
    [N,h1,w1,32] and FeatureNet's stage2 [N,16,2h1,2w1] / stage3 [N,8,4h1,4w1] (NCHW), differentiable
    w.r.t. all three and the four conv weights -> (stage2 [N,2h1,2w1,16], stage3 [N,4h1,4w1,8]) NHWC."""
    fp = model.FMT_with_pathway
    st2 = _PathwayStep.apply(stage1_nhwc, stage2_nchw, fp.dim_reduction_1.weight, fp.smooth_1.weight)
    st3 = _PathwayStep.apply(st2, stage3_nchw, fp.dim_reduction_2.weight, fp.smooth_2.weight)
    return st2, st3


_ENC_PARAMS = ("attention.query_projection.weight", "attention.query_projection.bias",
               "attention.key_projection.weight", "attention.key_projection.bias",
               "attention.value_projection.weight", "attention.value_projection.bias",
               "attention.out_projection.weight", "attention.out_projection.bias", "linear1.weight", "linear1.bias",
               "linear2.weight", "linear2.bias", "norm1.weight", "norm1.bias", "norm2.weight", "norm2.bias")


def _encoder_layer_backward(p, enc_w, x, src, dy, tpg, spg, self_attn):
    """EncoderLayer backward (models/FMT.py:96-111): x [T,32] the layer input, src [S,32] its attention
    source (x itself for a self layer), dy [T,32] -> (dx [T,32], dsrc [S,32] or None, 16 parameter grads).
    The token-wise forward is recomputed from x (HIP token kernels; K/V sums by the forward's own
    tmvs_fmt_kv); tpg / spg = query / source tokens per K/V group (a view for self layers; all views
    share the reference view's K/V in cross layers)."""
    wq, bq, wk, bk, wv, bv, wo, bo, w1, b1, w2, b2, g1, n1, g2, n2 = p
    groups = src.shape[0] // spg
    q = ops.token_linear(x, wq, bq)
    k = ops.token_linear(src, wk, bk)
    v = ops.token_linear(src, wv, bv)
    kv = ops.fmt_kv(src.view(groups, spg, 32), enc_w)
    msg = ops.linattn_fwd(q, kv, tpg)
    xp1 = ops.token_linear(msg, wo, bo, residual=x)                        # x + out_projection(msg)
    x1 = ops.layer_norm_fwd(xp1, g1, n1)
    hp = ops.token_linear(x1, w1, b1)
    hdn = ops.token_linear(x1, w1, b1, relu_of=hp)                         # relu(linear1(x1))
    xp2 = ops.token_linear(hdn, w2, b2, residual=x1)                       # x1 + linear2(hdn)
    dxp2, dgb2 = ops.layer_norm_bwd(dy, xp2, g2)
    dw2, db2 = ops.token_wgrad(dxp2, hdn)
    dhp = ops.token_linear(dxp2, w2, transpose_w=True, relu_of=hp)
    dw1, db1 = ops.token_wgrad(dhp, x1)
    dx1 = ops.token_linear(dhp, w1, transpose_w=True, residual=dxp2)
    dxp1, dgb1 = ops.layer_norm_bwd(dx1, xp1, g1)
    dwo, dbo = ops.token_wgrad(dxp1, msg)
    dmsg = ops.token_linear(dxp1, wo, transpose_w=True)
    dq, dkv = ops.linattn_bwd_q(q, dmsg, kv, tpg)
    dwq, dbq = ops.token_wgrad(dq, x)
    dx = ops.token_linear(dq, wq, transpose_w=True, out=dxp1)
    dk, dv = ops.linattn_bwd_kv(k, v, dkv, spg)
    dwk, dbk = ops.token_wgrad(dk, src)
    dwv, dbv = ops.token_wgrad(dv, src)
    dsrc = dx if self_attn else None
    dsrc = ops.token_linear(dk, wk, transpose_w=True, out=dsrc)
    ops.token_linear(dv, wv, transpose_w=True, out=dsrc)
    grads = (dwq, dbq, dwk, dbk, dwv, dbv, dwo, dbo, dw1, db1, dw2, db2, dgb1[:32], dgb1[32:], dgb2[:32], dgb2[32:])
    return dx, (None if self_attn else dsrc), grads


def _pack_enc(p):
    """The tmvs_fmt_* weight block of one layer from its 16 _ENC_PARAMS (as EncoderLayer.packed: key,
    value and linear2 weights transposed)."""
    parts = list(p)
    for i in (2, 4, 10):
        parts[i] = parts[i].t()
    return torch.cat([t.detach().float().contiguous().reshape(-1) for t in parts])


class _FMTTrain(torch.autograd.Function):
    """FMT (models/FMT.py:147-177, 212-220) for training: stage-1 features [nv,32,h,w] (reference view
    first) -> tokens [nv,h*w,32]. Forward: the inference kernels layer by layer (tmvs_fmt_embed,
    tmvs_fmt_kv, tmvs_fmt_apply), keeping each layer's input; backward: _encoder_layer_backward in
    reverse, the cross layers' source gradient summed into the reference view's tokens."""

    @staticmethod
    def forward(ctx, s1, pe, *params):
        nv, c, h, w = s1.shape
        L = h * w
        enc = gather_packs(list(params), [(tuple(range(16 * i, 16 * i + 16)), lambda *p: _pack_enc(p))
                                          for i in range(8)], "fmt_enc")  # one gather (packing.py)
        tokens = torch.empty(nv, L, c, device=s1.device)
        ops.fmt_embed(s1.contiguous(), pe, tokens)
        saved = []
        for j in range(4):
            xs = tokens.clone()
            ops.fmt_apply(tokens, ops.fmt_kv(tokens, enc[2 * j]), enc[2 * j])
            ref = tokens[0].clone()
            xc = tokens[1:].clone()
            ops.fmt_apply(tokens[1:], ops.fmt_kv(tokens[:1], enc[2 * j + 1]), enc[2 * j + 1], shared_kv=True)
            saved += [xs, ref, xc]
        ctx.save_for_backward(*saved, *params)
        ctx.enc, ctx.shape = enc, (nv, c, h, w)
        return tokens

    @staticmethod
    def backward(ctx, dtokens):
        nv, c, h, w = ctx.shape
        L = h * w
        t = ctx.saved_tensors
        saved, params = t[:12], [p.detach().float().contiguous() for p in t[12:]]
        grads = [None] * 128
        dt = dtokens.contiguous().clone()
        for j in reversed(range(4)):
            xs, ref, xc = saved[3 * j:3 * j + 3]
            i = 2 * j + 1
            dxc, dref, gi = _encoder_layer_backward(params[16 * i:16 * i + 16], ctx.enc[i], xc.view(-1, c), ref,
                                                    dt[1:].reshape(-1, c), (nv - 1) * L, L, False)
            dt[1:] = dxc.view(nv - 1, L, c)
            dt[0] += dref
            grads[16 * i:16 * i + 16] = gi
            i = 2 * j
            dxs, _, gi = _encoder_layer_backward(params[16 * i:16 * i + 16], ctx.enc[i], xs.view(-1, c), xs.view(-1, c),
                                                 dt.view(-1, c), L, L, True)
            dt = dxs.view(nv, L, c)
            grads[16 * i:16 * i + 16] = gi
        ds1 = dt.view(nv, h, w, c).permute(0, 3, 1, 2).contiguous()
        return (ds1, None, *grads)


def fmt_params(model):
    """The 128 FMT parameters (8 EncoderLayers x _ENC_PARAMS) in _FMTTrain's order."""
    layers = model.FMT_with_pathway.FMT.layers
    return [dict(layer.named_parameters())[n] for layer in layers for n in _ENC_PARAMS]


def fmt_train(model, stage1_nchw):
    """FMT_with_pathway's FMT part (models/FMT.py:212-220) for training: FeatureNet stage-1 features
    [nv,32,h,w] (reference view first) -> FMT output [nv,h,w,32] NHWC, differentiable w.r.t. the input
    and every FMT parameter (HIP forward and backward)."""
    if not stage1_nchw.is_cuda:
        raise RuntimeError("fmt_train runs on the GPU only (no CPU fallback)")
    nv, c, h, w = stage1_nchw.shape
    if nv < 2 or c != 32:
        raise ValueError("fmt_train: stage1 must be [nv >= 2, 32, h, w]")
    pe = model._pe_slice(h, w, stage1_nchw.device)
    tokens = _FMTTrain.apply(stage1_nchw, pe, *fmt_params(model))
    return tokens.view(nv, h, w, c)


def _pack_fwd(w, transposed):
    """Conv3d [Co][Ci][27] / ConvTranspose3d [Ci][Co][27] -> [27][Co][Ci]."""
    if transposed:
        ci, co = w.shape[:2]
        return w.reshape(ci, co, 27).permute(2, 1, 0).contiguous()
    co, ci = w.shape[:2]
    return w.reshape(co, ci, 27).permute(2, 0, 1).contiguous()


def _pack_dgrad(w, transposed):
    """The data-gradient conv maps Co -> Ci: [27][Ci][Co]."""
    if transposed:
        ci, co = w.shape[:2]
        return w.reshape(ci, co, 27).permute(2, 0, 1).contiguous()
    co, ci = w.shape[:2]
    return w.reshape(co, ci, 27).permute(2, 1, 0).contiguous()


def _fwd_pack_fn(cin, cout, stride, transposed):
    """The packing _conv_fwd's kernel reads: [27][Co][Ci], prob_kernel's [3][72] for the 8 -> 1 conv."""
    def fn(w):
        pk = _pack_fwd(w, transposed)
        return ops.prob_pack(pk) if not transposed and (cin, cout, stride) == (8, 1, 1) else pk
    return fn


def _dgrad_pack_fn(cin, cout, stride, transposed):
    """The packing _conv_dgrad's kernel reads (cin, cout: the forward layer's): [27][Ci][Co], its taps
    reversed for a stride-1 conv on the MFMA kernels (prob_kernel's packing for conv0's 8 -> 1)."""
    def fn(w):
        pk = _pack_dgrad(w, transposed)
        if not transposed and stride == 1 and (cout, cin, 1) in ops.MFMA_CONV:
            pk = pk.flip(0)
            if (cout, cin) == (8, 1):
                pk = ops.prob_pack(pk)
        return pk
    return fn


def _conv_fwd(x, pk, cout, odims, stride, transposed):
    """A CostRegNet layer's raw convolution (before train-mode BN) with pk = _fwd_pack_fn's packing: the
    inference layers' MFMA kernels (tmvs_conv3d_mfma) where they cover the (cin, cout, stride), else
    tmvs_conv3d_generic."""
    cin = x.shape[-1]
    if (cin, cout) in ops.MFMA_DECONV if transposed else (cin, cout, stride) in ops.MFMA_CONV:
        return ops.conv3d_mfma(x, pk, cout, stride, transposed)
    return ops.conv3d_generic(x, pk, cout, odims, stride, transposed)


def _conv_dgrad(dz, pk, cin, idims, stride, transposed, acc):
    """d input of a layer (+ acc, the gradient already gathered for that tensor through a skip), pk =
    _dgrad_pack_fn's packing:
      ConvTranspose3d -> Conv3d stride 2 of dz with the same weight tensor read as [Ci_t][Co_t];
      Conv3d stride 2 -> ConvTranspose3d of dz with the weight read as ConvTranspose [Co][Ci];
      Conv3d stride 1 -> Conv3d of dz with the taps reversed and [Co][Ci] transposed.
    On the MFMA kernels where they cover the shape, else the generic gathers."""
    cout = dz.shape[-1]
    if transposed and (cout, cin, 2) in ops.MFMA_CONV:
        dx = ops.conv3d_mfma(dz, pk, cin, 2)
    elif not transposed and stride == 2 and (cout, cin) in ops.MFMA_DECONV:
        return ops.conv3d_mfma(dz, pk, cin, 2, transposed=True, skip=acc)
    elif not transposed and stride == 1 and (cout, cin, 1) in ops.MFMA_CONV:
        dx = ops.conv3d_mfma(dz, pk, cin, 1)
    elif transposed:  # strided gather of dz
        return ops.conv3d_generic(dz, pk, cin, idims, 2, False, out=acc)
    else:  # transposed gather of dz
        return ops.conv3d_generic(dz, pk, cin, idims, stride, True, out=acc)
    if acc is None:
        return dx
    return acc.add_(dx)


def _layer_channels(w, transposed):
    """(cin, cout) of a Conv3d [Co][Ci][..] / ConvTranspose3d [Ci][Co][..] weight."""
    return (w.shape[0], w.shape[1]) if transposed else (w.shape[1], w.shape[0])


def _unpack_wgrad(dw27, shape):
    """[27][A][B] -> the torch weight layout [A][B][3][3][3] (A, B = Co, Ci or Ci, Co)."""
    return dw27.permute(1, 2, 0).reshape(shape).contiguous()


def _down(dhw):
    return tuple((n - 1) // 2 + 1 for n in dhw)


class _CostRegNetTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eps, stats_out, *params):
        b, d, h, w = x.shape
        ws = params[:-1]
        wprob = params[-1]
        # every layer's forward and data-gradient packings in one gather (packing.py)
        weights = [ws[3 * i] for i in range(len(_LAYERS))] + [wprob]
        geo = [(i, *_layer_channels(weights[i], tr), st, tr) for i, (_, st, tr, _) in enumerate(_LAYERS)]
        geo.append((len(_LAYERS), 8, 1, 1, False))
        packs = gather_packs(weights, [(i, _fwd_pack_fn(ci, co, st, tr)) for i, ci, co, st, tr in geo] +
                             [(i, _dgrad_pack_fn(ci, co, st, tr)) for i, ci, co, st, tr in geo], "costregnet")
        fwd_pk, ctx.dgrad_pk = packs[:len(geo)], packs[len(geo):]
        acts = {"input": (x.contiguous().view(b, d, h, w, 1), (d, h, w))}
        saved = []
        cur, dims = acts["input"]
        stats = []
        for i, (name, stride, transposed, skip) in enumerate(_LAYERS):
            wt, g, bt = ws[3 * i], ws[3 * i + 1], ws[3 * i + 2]
            cout = wt.shape[1] if transposed else wt.shape[0]
            odims = tuple(2 * n for n in dims) if transposed else (dims if stride == 1 else _down(dims))
            z = _conv_fwd(cur, fwd_pk[i], cout, odims, stride, transposed)
            mean, var = ops.bn_stats(z)
            y = ops.bn_relu_train(z, mean, var, g.detach(), bt.detach(), eps,
                                  skip=acts[skip][0] if skip is not None else None)
            saved.append((cur, dims, z, mean, var))
            stats.append((mean, var, z.numel() // z.shape[-1]))
            acts[name] = (y, odims)
            cur, dims = y, odims
        logits = _conv_fwd(cur, fwd_pk[-1], 1, dims, 1, False)
        ctx.eps = eps
        ctx.layer_io = saved
        ctx.u11 = cur
        stats_out.extend(stats)
        ctx.save_for_backward(*params)
        return logits.view(b, d, h, w)

    @staticmethod
    def backward(ctx, dlogits):
        params = ctx.saved_tensors
        ws, wprob = params[:-1], params[-1]
        eps = ctx.eps
        b, d, h, w = dlogits.shape
        g = dlogits.contiguous().view(b, d, h, w, 1)
        grads = [None] * len(params)
        dws = [None] * (len(_LAYERS) + 1)
        dws[-1] = ops.conv3d_wgrad(g, ctx.u11, 1)
        # gradient w.r.t. each layer's output, filled as the backward reaches it
        dout = {"conv11": _conv_dgrad(g, ctx.dgrad_pk[-1], ctx.u11.shape[-1], (d, h, w), 1, False, None)}
        for i in range(len(_LAYERS) - 1, -1, -1):
            name, stride, transposed, skip = _LAYERS[i]
            wt, gm, bt = ws[3 * i], ws[3 * i + 1], ws[3 * i + 2]
            xin, idims, z, mean, var = ctx.layer_io[i]
            dy = dout.pop(name)
            if skip is not None:  # y = skip + relu(bn(z)): the skip source receives dy as is (aliased: dy is
                # only read again by bn_relu_backward below, stream-ordered before any in-place accumulation)
                dout[skip] = dy if skip not in dout else dout[skip].add_(dy)
            dz, dgam, dbet = ops.bn_relu_backward(dy, z, mean, var, gm.detach(), bt.detach(), eps)
            if transposed:
                dw = ops.conv3d_wgrad(xin, dz, 2)
            else:
                dw = ops.conv3d_wgrad(dz, xin, stride)
            dws[i] = dw
            grads[3 * i + 1], grads[3 * i + 2] = dgam, dbet
            prev = _LAYERS[i - 1][0] if i > 0 else "input"
            cin = xin.shape[-1]
            acc = dout.get(prev)
            dout[prev] = _conv_dgrad(dz, ctx.dgrad_pk[i], cin, idims, stride, transposed, acc)
        # the weight gradients back to the torch layouts, one gather for all layers
        shapes = [ws[3 * i].shape for i in range(len(_LAYERS))] + [wprob.shape]
        unp = gather_packs(dws, [(i, (lambda t, s=s_: _unpack_wgrad(t, s))) for i, s_ in enumerate(shapes)],
                           "costregnet_wgrad")
        for i in range(len(_LAYERS)):
            grads[3 * i] = unp[i]
        grads[-1] = unp[-1]
        ctx.dgrad_pk = None
        dx = dout["input"].view(b, d, h, w)
        return (dx, None, None, *grads)


def costregnet_params(module):
    """The tensors _CostRegNetTrain differentiates, in its order: per layer (conv weight, BN gamma,
    BN beta), then prob.weight."""
    ps = []
    for name, _, _, _ in _LAYERS:
        blk = getattr(module, name)
        ps += [blk.conv.weight, blk.bn.weight, blk.bn.bias]
    return ps + [module.prob.weight]


def costregnet_train(module, x):
    """CostRegNet.forward in train mode on the HIP kernels; differentiable w.r.t. x and the module's
    parameters; updates the BatchNorm running statistics like nn.BatchNorm3d (momentum 0.1)."""
    if not x.is_cuda:
        raise RuntimeError("costregnet_train runs on the GPU only (no CPU fallback)")
    if x.dim() != 4 or any(n % 8 for n in x.shape[1:]):
        raise ValueError("costregnet_train: x must be [B, D, H, W] with D, H, W divisible by 8")
    eps = module.conv0.bn.eps
    params = costregnet_params(module)
    stats = []
    with torch.cuda.device(x.device):
        logits = _CostRegNetTrain.apply(x.float(), eps, stats, *params)
        update_running_stats([(getattr(module, name).bn, mean[None], var[None], n)
                              for (name, _, _, _), (mean, var, n) in zip(_LAYERS, stats)], BN_MOMENTUM)
    return logits


class _AggregateTrain(torch.autograd.Function):
    """View aggregation (TransMVSNet.py:71-93) with, at stage 1, the train-mode PixelwiseNet weights
    (TransMVSNet.py:10-30), forward and backward on csrc/pw_train.hip. Outputs (sim [D,H,W], the
    view weights used [V,H',W'], non-differentiable as the reference returns them detached)."""

    @staticmethod
    def forward(ctx, sims, pwp, vw_given, vw_shift, stats_out):
        sims = sims.contiguous()
        if vw_given is None:
            stats, vw, dstar = ops.pixelwise_train_forward(sims, pwp.detach().contiguous())
            stats_out.append(stats)
            ctx.pw = (stats, dstar)
        else:
            vw = vw_given.contiguous()
            ctx.pw = None
        sim, wsum = ops.aggregate_train(sims, vw, vw_shift)
        ctx.vw_shift = vw_shift
        ctx.save_for_backward(sims, sim, wsum, vw, pwp)
        ctx.mark_non_differentiable(vw)
        return sim, vw

    @staticmethod
    def backward(ctx, dsim, _dvw):
        sims, sim, wsum, vw, pwp = ctx.saved_tensors
        stage1 = ctx.pw is not None
        dsims, dvw = ops.aggregate_train_backward(dsim.contiguous(), sims, sim, wsum, vw, ctx.vw_shift, stage1)
        dpwp = None
        if stage1:
            stats, dstar = ctx.pw
            dpwp = ops.pixelwise_train_backward(sims, pwp.detach().contiguous(), stats, vw, dstar, dvw, dsims)
        return dsims, dpwp, None, None, None


def _pw_params(pw):
    """The 201-float device parameter block of tmvs_pixelwise_train_* (differentiable torch.cat)."""
    return torch.cat([pw.conv0.conv.weight.reshape(16), pw.conv0.bn.weight, pw.conv0.bn.bias,
                      pw.conv1.conv.weight.reshape(128), pw.conv1.bn.weight, pw.conv1.bn.bias,
                      pw.conv2.weight.reshape(8), pw.conv2.bias.reshape(1)]).float()


def aggregate_train(sims, model, vw_given=None, vw_shift=0):
    """DepthNet's view aggregation for training; at stage 1 (vw_given None) the view weights come
    from PixelwiseNet in train mode, whose BatchNorm running statistics are updated once per view
    (the reference calls it per view). Returns (sim [D,H,W], view weights)."""
    pw = model.DepthNet.pixel_wise_net
    stats = []
    sim, vw = _AggregateTrain.apply(sims, _pw_params(pw), vw_given, vw_shift, stats)
    if stats:
        n = sims.shape[1] * sims.shape[2] * sims.shape[3]
        st = torch.stack(list(stats[0]))  # [views, 48], views in order
        update_running_stats([(pw.conv0.bn, st[:, 0:16], st[:, 16:32], n), (pw.conv1.bn, st[:, 32:40], st[:, 40:48], n)],
                             pw.conv0.bn.momentum)
    return sim, vw


class _SoftmaxWTA(torch.autograd.Function):
    """prob = exp(log_softmax(logits)), depth / confidence by WTA (models/TransMVSNet.py:97-103,
    217-221) on tmvs_softmax_wta; the backward of prob is tmvs_softmax_backward (depth, the raw
    depth and the confidence carry no gradient, as in the reference)."""

    @staticmethod
    def forward(ctx, logits, hyp):
        from .model import DEPTH_CLAMP
        prob, depth, raw, conf = ops.softmax_wta(logits.detach().contiguous(), hyp, DEPTH_CLAMP)
        ctx.save_for_backward(prob)
        ctx.mark_non_differentiable(depth, raw, conf)
        return prob, depth, raw, conf

    @staticmethod
    def backward(ctx, dprob, _d, _r, _c):
        if dprob is None:
            return None, None
        (prob,) = ctx.saved_tensors
        return ops.softmax_backward(prob, dprob.contiguous()), None


def depth_stages_forward_train(model, stage_features, proj_matrix, depth_values, img_hw):
    """The three DepthNet stages of a training forward for ONE sample (B = 1): TransMVSNet.forward's
    stage loop (models/TransMVSNet.py:168-221) in train mode, returning its output dict (per stage
    depth / photo_confidence / prob_volume / depth_values, plus the stage-3 keys at the top level).
    prob_volume is differentiable (through the HIP softmax, CostRegNet, aggregation / PixelwiseNet
    and cost-volume backward into the stage features); each prob_volume also carries its logits as
    `_tmvs_logits`, so transmvsnet_amd.loss can seed the backward with d loss / d logits directly.

    stage_features: {stage: [N, h, w, C]} NHWC FMT/pathway outputs, reference view first; proj_matrix
    {stage: [1, N, 2, 4, 4]}; depth_values [1, 192]. The CostRegNets and the PixelwiseNet run in
    train mode (their BatchNorm running statistics are updated)."""
    from .model import STAGE_SCALES
    dev = stage_features["stage1"].device
    with torch.cuda.device(dev):
        dv = depth_values.to(dev, torch.float32).contiguous()
        outputs, prev_raw, vw_det = {}, None, None
        for s in range(3):
            name = f"stage{s + 1}"
            f = stage_features[name]
            hyp = ops.stage_hypotheses(dv, prev_raw, model.ndepths[s], model.depth_interals_ratio[s], img_hw,
                                       STAGE_SCALES[s])
            rows = ops.proj_rows(proj_matrix[name])[0]
            sims = warp_corr_views(f[0], f[1:], hyp[0], rows, rot_order=model.warp_rot_order,
                                   planes=prev_raw is None)  # [V,D,h,w]; stage 1: depth planes
            if s == 0:  # TransMVSNet.py:107 returns the stage-1 view weights detached
                sim, vw_det = aggregate_train(sims, model)
            else:       # nearest x2 per stage (:194) = reading the stage-1 map at (y >> s, x >> s)
                sim, _ = aggregate_train(sims, model, vw_det, s)
            logits = costregnet_train(model.cost_regularization[s].train(), sim.unsqueeze(0))
            prob, depth, raw, conf = _SoftmaxWTA.apply(logits, hyp)
            prob._tmvs_logits = logits
            outputs[name] = {"depth": depth, "photo_confidence": conf, "prob_volume": prob, "depth_values": hyp}
            outputs.update(outputs[name])
            prev_raw = raw
    return outputs


def depth_stages_train(model, stage_features, proj_matrix, depth_values, depth_gt_ms, mask_ms, img_hw,
                       dlossw=(0.5, 1.0, 2.0), loss="trans_mvsnet", depth_interval=None):
    """One training step's DepthNet stages for ONE sample (B = 1), forward and backward.

    stage_features: {stage: [N, h, w, C]} NHWC FMT/pathway outputs, reference view first (leaf tensors
    that require grad collect d loss / d features); proj_matrix {stage: [1, N, 2, 4, 4]}; depth_values
    [1, 192]; depth_gt_ms / mask_ms {stage: [1, h, w]}. The CostRegNets and the PixelwiseNet run in train
    mode (their BatchNorm running statistics are updated). Calls backward of the loss and returns
    (total_loss, outputs) with outputs as TransMVSNet.forward's stage dicts. loss="trans_mvsnet":
    train.py:152's trans_mvsnet_loss (dlossw default 0.5,1,2); loss="focal_bld": finetune.py:159's
    focal_loss_bld for BlendedMVS (config C5; pass dlossw=(1, 1, 1), finetune.py:42, and the sample's
    depth_interval) -- outputs["metrics"] then holds its (depth_loss, epe, less1, less3).
    """
    if loss not in ("trans_mvsnet", "focal_bld"):
        raise ValueError(f"depth_stages_train: loss must be 'trans_mvsnet' or 'focal_bld', got {loss!r}")
    if loss == "focal_bld" and depth_interval is None:
        raise ValueError("depth_stages_train: focal_bld needs depth_interval")
    from . import loss as loss_mod
    dev = stage_features["stage1"].device
    with torch.cuda.device(dev):
        outputs = depth_stages_forward_train(model, stage_features, proj_matrix, depth_values, img_hw)
        logits_all = [outputs[f"stage{s + 1}"]["prob_volume"]._tmvs_logits for s in range(3)]
        with torch.no_grad():
            if loss == "focal_bld":
                total, depth_loss, epe, less1, less3, grads = loss_mod.focal_loss_bld(
                    outputs, depth_gt_ms, mask_ms, depth_interval, dlossw=dlossw, return_grad=True)
                outputs["metrics"] = {"depth_loss": depth_loss, "epe": epe, "less1": less1, "less3": less3}
            else:
                total, depth_loss, _, _, grads = loss_mod.trans_mvsnet_loss(outputs, depth_gt_ms, mask_ms,
                                                                            dlossw=dlossw, return_grad=True)
        global _DEFERRED_FLAGS
        _DEFERRED_FLAGS = []
        try:
            torch.autograd.backward(logits_all, [grads[f"stage{s + 1}"] for s in range(3)])
            flags = _DEFERRED_FLAGS
        finally:
            _DEFERRED_FLAGS = None
        if torch.cuda.is_current_stream_capturing():
            GRAPH_FLAGS.extend(_sticky_flag(f) for f in flags)
        else:
            _check_overflow(flags)
    return total, outputs


def forward_train(model, imgs, proj_matrix, depth_values):
    """TransMVSNet.forward (models/TransMVSNet.py:141-226) in train mode, on HIP: FeatureNet
    (featurenet_train), the FMT (fmt_train), FMT_with_pathway's lateral steps (pathway_train) and the
    three DepthNet stages (depth_stages_forward_train), every block differentiable through its HIP
    backward, so the reference's train_sample body (finetune.py:144-168) runs unchanged:
    ``model.train(); outputs = model(imgs, proj, dv); loss = focal_loss_bld(outputs, ...)[0];
    loss.backward(); optimizer.step()``. One sample per call (B = 1: C5's DDP runs one sample per
    rank, finetune.py batch_size 1 per process)."""
    from .featurenet_train import featurenet_train
    if imgs.dim() != 5 or imgs.shape[0] != 1:
        raise ValueError("TransMVSNet train-mode forward takes one sample per call: imgs [1, N, 3, H, W]")
    if not imgs.is_cuda:
        raise RuntimeError("TransMVSNet (HIP) needs GPU inputs; the HIP path has no CPU fallback")
    h, w = imgs.shape[3], imgs.shape[4]
    with torch.cuda.device(imgs.device):
        s1, s2, s3 = featurenet_train(model.feature, imgs[0])
        st1 = fmt_train(model, s1)
        st2, st3 = pathway_train(model, st1, s2, s3)
        return depth_stages_forward_train(model, {"stage1": st1, "stage2": st2, "stage3": st3}, proj_matrix,
                                          depth_values, (h, w))


class FlatAdam:
    """torch.optim.Adam as finetune.py:324 builds it (lr, betas=(0.9, 0.999), eps=1e-8, L2 weight_decay),
    over ONE flat fp32 buffer: at construction every parameter's storage becomes a view of `flat`.
    Gradients are left to autograd (no per-parameter accumulate kernels): `zero_grad` sets them to
    None, and the first of `allreduce` / `step` gathers them into `grad_flat` with one concatenation,
    re-pointing each .grad at its slice. The DDP sync is then one all-reduce of `grad_flat`, and a
    step is one HIP launch (tmvs_adam_step)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("FlatAdam: no parameters")
        dev = self.params[0].device
        if any(p.device != dev or p.dtype != torch.float32 for p in self.params):
            raise ValueError("FlatAdam: every parameter must be float32 on one device")
        if len({id(p) for p in self.params}) != len(self.params):
            raise ValueError("FlatAdam: a parameter is listed twice")
        n = sum(p.numel() for p in self.params)
        self.flat = torch.empty(n, device=dev)
        self.grad_flat = torch.zeros(n, device=dev)
        self._segs, off = [], 0
        for p in self.params:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            self._segs.append((off, k))
            off += k
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self._host_steps = 0
        self._graphed = False
        # the step number on the device as well, for a step captured in a HIP graph (tmvs_adam_step_dev
        # advances it per replay); eager steps before any capture keep it equal to the host count
        self._step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self._scal_dev = torch.zeros(2, device=dev)
        # the learning rate a captured step reads when it runs (tmvs_adam_step_dev lr_dev): sync_lr writes
        # self.lr there before each replay (TrainStepGraph.replay does), so a schedule that sets opt.lr
        # per iteration (finetune.py:58-72, WarmupMultiStepLR) holds under replays too
        self._lr_dev = torch.full((1,), float(lr), dtype=torch.float64, device=dev)
        self._lr_dev_val = float(lr)
        self._gathered = False

    def sync_lr(self, lr=None):
        """Write lr (default self.lr) to the device scalar a captured step reads (outside a capture)."""
        lr = float(self.lr if lr is None else lr)
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("FlatAdam.sync_lr: call outside a HIP-graph capture (before replaying)")
        if lr != self._lr_dev_val:
            self._lr_dev.fill_(lr)
            self._lr_dev_val = lr

    def zero_grad(self):
        for p in self.params:
            p.grad = None
        self._gathered = False

    def _is_slice(self, p, off):
        """p.grad is still the grad_flat view `_gather` installed (a later backward accumulated
        into it in place)."""
        g = p.grad
        return (g is not None and g.data_ptr() == self.grad_flat.data_ptr() + 4 * off
                and g.is_contiguous() and g.shape == p.shape)

    def _gather(self):
        if self._gathered:
            return
        slices = [self._is_slice(p, off) for p, (off, _) in zip(self.params, self._segs)]
        # a .grad that is not already its grad_flat view (after a first backward: all of them; with
        # gradient accumulation over several backwards: only those autograd replaced) is copied in
        # with multi-tensor launches; parameters without a gradient get zeros
        dst, src, none = [], [], []
        for p, (off, k), inside in zip(self.params, self._segs, slices):
            if inside:
                continue
            if p.grad is None:
                none.append(self.grad_flat[off:off + k])
            else:
                dst.append(self.grad_flat[off:off + k])
                src.append(p.grad.reshape(-1))
        if none:
            if not any(slices) and len(none) > 8:
                self.grad_flat.zero_()
            else:
                torch._foreach_zero_(none)
        if dst:
            torch._foreach_copy_(dst, src)
        for p, (off, k) in zip(self.params, self._segs):
            p.grad = self.grad_flat[off:off + k].view_as(p)
        self._gathered = True

    def allreduce(self, group=None):
        """DDP's gradient mean over ranks: one all_reduce(SUM) of the flat gradient, then 1/world."""
        import torch.distributed as dist
        self._gather()
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(self.grad_flat, op=dist.ReduceOp.SUM, group=group)
            self.grad_flat.div_(dist.get_world_size(group))

    @property
    def step_count(self):
        """Adam's step number. Once a step has been captured in a HIP graph, replays advance only the
        device counter, so that counter is the only count from then on (one host sync to read)."""
        return int(self._step_dev.item()) if self._graphed else self._host_steps

    def step(self, lr=None):
        self._gather()
        lr = self.lr if lr is None else lr
        capturing = torch.cuda.is_current_stream_capturing()
        if capturing or self._graphed:
            # captured (the launch runs once per replay) or any step after a capture: the step number
            # lives on the device (tmvs_adam_step_dev advances it per launch); the host count is not
            # touched, so eager steps interleaved with replays use the right bias correction. The
            # learning rate is read from _lr_dev when the launch runs: a captured step takes the value
            # sync_lr wrote before the replay (CAPTURED_OPTIMIZERS lets TrainStepGraph find this
            # optimizer); an eager step writes its own lr first.
            self._graphed = True
            if capturing:
                # an explicit lr becomes the optimizer's: TrainStepGraph.replay syncs opt.lr into _lr_dev before
                # every replay, so the captured step keeps applying it (a raw torch.cuda.graph replay must call
                # sync_lr itself: the launch reads whatever _lr_dev holds)
                self.lr = lr
                if _TSG_CAPTURES:
                    CAPTURED_OPTIMIZERS.append(self)
            else:
                self.sync_lr(lr)
            ops.adam_step_dev(self.flat, self.grad_flat, self.exp_avg, self.exp_avg_sq, lr, self.betas, self.eps,
                              self.weight_decay, self._step_dev, self._scal_dev, lr_dev=self._lr_dev)
        else:
            self._host_steps += 1
            ops.adam_step(self.flat, self.grad_flat, self.exp_avg, self.exp_avg_sq, lr, self.betas, self.eps,
                          self.weight_decay, self._host_steps)
            self._step_dev.fill_(self._host_steps)
        # the launch wrote the parameters through a raw pointer: bump their version counters so the
        # inference caches keyed on them (TransMVSNet._param_key, FeatureNet's packed weights) rebuild
        # (a replay bumps nothing: TrainStepGraph.replay does it)
        bump_versions(self.params)
        self._gathered = False  # the next backward adds into the current .grad views unless zero_grad runs


def bump_versions(tensors):
    """Advance the in-place version counter of every tensor (after a raw-pointer write or a graph replay
    that wrote them), so caches keyed on `_version` rebuild."""
    with torch.no_grad():
        for t in tensors:
            torch.autograd.graph.increment_version(t)


CAPTURED_OPTIMIZERS = []  # FlatAdams whose step a TrainStepGraph captured (it syncs their lr per replay)
_TSG_CAPTURES = []  # non-empty while a TrainStepGraph captures


class TrainStepGraph:
    """A training step captured once as a HIP graph and replayed (finetune.py:144-168's body per replay).

    * The overflow flags of the warp backwards captured in this graph are kept per graph as sticky
      words (every replay ORs its flags in) and checked by `check_flags`, which raises if any replay
      since the last check overflowed and then clears them; one graph's overflow never blocks
      another's check.
    * The learning rate of a FlatAdam step captured in the graph is read from the device when the
      replay runs: `replay` first writes each such optimizer's current `lr` there (FlatAdam.sync_lr),
      so a per-iteration schedule (finetune.py:58-72) is followed.
    * `replay` bumps the version counters of the model's parameters and buffers (the replay's Adam step
      and BatchNorm running-statistic updates wrote them without Python seeing it), so an eval forward
      after replays rebuilds the inference caches (TransMVSNet._param_key, FeatureNet's packed
      weights) instead of running on the weights of the last eager step.
    Index caches that a step fills lazily (packing.gather_packs, featurenet_train's pack indices) must
    be warm before capture: run the step once eagerly first (capture raises otherwise)."""

    def __init__(self, fn, model, stream=None):
        self.model = model
        self.graph = torch.cuda.CUDAGraph()
        dev = next(model.parameters()).device
        reserve_graph_flags(dev, 64)
        n0, o0 = len(GRAPH_FLAGS), len(CAPTURED_OPTIMIZERS)
        _TSG_CAPTURES.append(self)
        try:
            with torch.cuda.graph(self.graph, stream=stream):
                self.out = fn()
            self.flags = GRAPH_FLAGS[n0:]
            self.optimizers = list(dict.fromkeys(CAPTURED_OPTIMIZERS[o0:]))
        finally:  # a failed capture leaves nothing behind
            _TSG_CAPTURES.pop()
            del GRAPH_FLAGS[n0:]
            del CAPTURED_OPTIMIZERS[o0:]
        self._tensors = list(model.parameters()) + list(model.buffers())

    def replay(self):
        for opt in self.optimizers:
            opt.sync_lr()
        self.graph.replay()
        bump_versions(self._tensors)
        return self.out

    def check_flags(self):
        """One host sync: raise if any captured warp backward overflowed in any replay since the last
        check; the sticky flags are cleared afterwards."""
        try:
            _check_overflow(self.flags)
        finally:
            for f in self.flags:
                f.zero_()


def allreduce_gradients(params, group=None, bucket_bytes=64 << 20):
    """DDP's gradient synchronisation (train.py:363-366 wraps the model in DistributedDataParallel):
    the mean over ranks of every parameter gradient, as few flat buckets (one at this model's
    4.6 MB) reduced with one all_reduce(SUM) each over RCCL, then scaled by 1/world."""
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return
    world = dist.get_world_size(group)
    grads = [p.grad for p in params if p.grad is not None]
    if world == 1 or not grads:
        return
    bucket, size = [], 0
    for g in grads + [None]:
        if g is not None and size + g.numel() * 4 <= bucket_bytes or (g is not None and not bucket):
            bucket.append(g)
            size += g.numel() * 4
            continue
        flat = torch.cat([b.reshape(-1) for b in bucket])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        flat.div_(world)
        off = 0
        for b in bucket:
            b.copy_(flat[off:off + b.numel()].view_as(b))
            off += b.numel()
        if g is not None:
            bucket, size = [g], g.numel() * 4
