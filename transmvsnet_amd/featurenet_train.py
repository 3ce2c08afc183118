"""FeatureNet in train mode with its backward on HIP.

``featurenet_train(fnet, imgs)`` is FeatureNet.forward (models/module.py:399-422) of one sample's N
views [N,3,H,W] with every BatchNorm in train mode, as the reference runs it inside train_sample
(finetune.py:144-168: ``model.train()``; the reference calls FeatureNet once per view,
models/TransMVSNet.py:151-153, so batch statistics are per view and each BatchNorm's running
statistics are updated once per view, in view order, momentum 0.1, unbiased variance). Returns the
stage features NCHW (stage1 [N,32,H/4,W/4], stage2 [N,16,H/2,W/2], stage3 [N,8,H,W]),
differentiable w.r.t. every FeatureNet parameter (the image needs no gradient).

Forward: the inference kernels without their folded BatchNorm -- tmvs_conv2d_bn_relu (trunk and the
stage-1 head's 1x1), tmvs_conv3x3_nhwc (stage-2/3 heads' 3x3), tmvs_fpn_merge, and each DCN as ONE
tmvs_dcn_forward_train launch (offset/mask conv + deformable conv, also writing the offset/mask
tensor for the backward) -- then tmvs_bn_stats_grouped / tmvs_bn_relu_train_grouped (group = view).
Backward (csrc/featurenet_train.hip + the BatchNorm kernels of costreg_train.hip): per layer in
reverse, tmvs_bn_relu_backward_grouped (group = view), weight gradients tmvs_conv2d_wgrad, data gradients
tmvs_conv2d_generic (transposed gathers), the DCN by tmvs_dcn_backward (dcol, d offsets / d mask
logits, dW, the bilinear scatter into dx) followed by its offset/mask conv's gradients, bias
gradients tmvs_colsum, the FPN merges' nearest x2 adjoint tmvs_nearest_up2_backward_nhwc.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import ops
from .bn_running import update_running_stats
from .packing import gather_packs

BN_MOMENTUM = 0.1
_PACK_INDEX = {}


def _pack_index(kind, cout, cin, k, device):
    """Flat gather indices reproducing the host packers tmvs_deform_conv2d_pack / tmvs_conv2d_pack
    (csrc/featurenet.hip, csrc/conv2d.hip) into a weight flattened [cout][cin][k*k] plus one trailing
    zero (index cout*cin*k*k = a padding slot), so training packs on the device with no host sync."""
    key = (kind, cout, cin, k, str(device))
    if key not in _PACK_INDEX:
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            # the host-to-device copy below cannot run inside a capture (and would cache garbage)
            raise RuntimeError(f"featurenet_train: pack index {key[:4]} not built yet inside a HIP-graph "
                               "capture; run the step once eagerly before capturing it")
        zero = cout * cin * k * k
        if kind == "dcn":  # [tap][m-tile][half][lane][e] <- W[16m + (l & 15)][16h + 4 (l >> 4) + e][tap]
            mt = (cout + 15) // 16
            t, m, h, lane, e = np.meshgrid(np.arange(9), np.arange(mt), np.arange(2), np.arange(64), np.arange(4),
                                           indexing="ij")
            co, ci = 16 * m + (lane & 15), 16 * h + 4 * (lane >> 4) + e
            idx = np.where(co < cout, (co * cin + ci) * 9 + t, zero)
        else:  # conv2d: the host packer itself on an index-valued weight (value i + 1 at flat index i; a
            # packed 0 is a padding slot), so the layout -- incl. the 8-channel row-pair form -- is the C one
            from . import ops
            w_idx = torch.arange(1, zero + 1, dtype=torch.float32).reshape(cout, cin, k, k)  # exact below 2^24
            packed = ops.conv2d_pack(w_idx).numpy().astype(np.int64)
            idx = np.where(packed > 0, packed - 1, zero)
        _PACK_INDEX[key] = torch.from_numpy(idx.reshape(-1).astype(np.int64)).to(device)
    return _PACK_INDEX[key]


def _offset_dgrad_index(device):
    """Gather indices from conv_offset_mask.weight [27][32][3][3] (flattened, plus one trailing zero)
    straight to the 'dcn' pack of its data-gradient weight: the weight zero-padded to 32 output rows,
    flipped in both spatial axes and transposed (in <-> out), as dgrad_same builds it -- one gather
    instead of the pad, flip, transpose and pack launches."""
    key = ("offdgrad", str(device))
    if key not in _PACK_INDEX:
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("featurenet_train: offset-conv dgrad index not built yet inside a HIP-graph "
                               "capture; run the step once eagerly before capturing it")
        zero = 27 * 32 * 9
        a, b, kh, kw = np.meshgrid(np.arange(32), np.arange(32), np.arange(3), np.arange(3), indexing="ij")
        # flipped-transposed padded weight wf[a][b][kh][kw] = W[b][a][2 - kh][2 - kw] (0 for b >= 27)
        src = np.where(b < 27, ((b * 32 + a) * 3 + (2 - kh)) * 3 + (2 - kw), zero).reshape(-1)
        src = np.concatenate([src, [zero]])
        pidx = _pack_index("dcn", 32, 32, 3, "cpu").numpy()
        _PACK_INDEX[key] = torch.from_numpy(src[pidx].astype(np.int64)).to(device)
    return _PACK_INDEX[key]


def offset_dgrad_pack(w_offset_mask):
    """device_pack('dcn', _flip_t(W zero-padded to 32 rows)) of conv_offset_mask.weight, one gather."""
    flat = torch.cat([w_offset_mask.detach().float().reshape(-1),
                      w_offset_mask.new_zeros(1, dtype=torch.float32)])
    return flat[_offset_dgrad_index(w_offset_mask.device)]


def device_pack(kind, w):
    """The kernels' packed weight layout, gathered on the weight's device ('dcn' or 'conv2d')."""
    co, ci, k, _ = w.shape
    flat = torch.cat([w.detach().float().reshape(-1), w.new_zeros(1, dtype=torch.float32)])
    return flat[_pack_index(kind, co, ci, k, w.device)].contiguous()


# ------------------------------------------------------------------------- the step's weight packs
# Every weight re-layout a FeatureNet step needs (forward packs, data-gradient packs, tap transposes) is
# gathered ONCE per forward by _prepare_packs (packing.gather_packs: one cat + one index gather instead of
# ~130 small cat / index / flip / permute launches); the layer functions look their packs up in the active
# table and fall back to packing on the spot for a weight not in it. Each forward's table is kept on its
# autograd context and made active again for its own backward (_active_packs), so a backward always uses the
# packs of the weights its forward ran with, whatever other forwards ran in between.
_STEP_PACKS = {}


def _pk(key):
    return _STEP_PACKS.get(key)


class _active_packs:
    """with _active_packs(table): the layer functions' _pk lookups read `table` (restored on exit)."""

    def __init__(self, table):
        self.table = table

    def __enter__(self):
        global _STEP_PACKS
        self.prev, _STEP_PACKS = _STEP_PACKS, self.table

    def __exit__(self, *a):
        global _STEP_PACKS
        _STEP_PACKS = self.prev


def _pack_fn(kind, co, ci, k):
    return lambda t: torch.cat([t.reshape(-1), t.new_zeros(1)])[_pack_index(kind, co, ci, k, t.device)]


def _dgrad_kind(co, ci, k):
    """The data-gradient form dgrad_same takes for a stride-1 conv weight [co][ci][k][k]."""
    if ci == 32 and co == 32 and k == 3:
        return "dcn"
    if (co, ci, k) in _MFMA_DGRAD:
        return "conv2d"
    return "taps_t"


def _prepare_packs(fnet):
    """A new pack table (one gather_packs call for the whole FeatureNet) made active for the forward
    (TMVS_NO_STEP_PACKS=1: empty -- every layer packs on the spot, the previous form; for bitwise A/Bs)."""
    global _STEP_PACKS
    table = _STEP_PACKS = {}
    if os.environ.get("TMVS_NO_STEP_PACKS") == "1":
        return table
    tensors, specs, keys = [], [], []

    def add(t, fn, key):
        tensors.append(t)
        specs.append((len(tensors) - 1, fn))
        keys.append(key)

    def block(blk, k, stride, head3x3=False, need_dx=True):
        w = blk.conv.weight
        co, ci = w.shape[0], w.shape[1]
        add(w, _pack_fn("dcn" if head3x3 else "conv2d", co, ci, k), ("fwd", id(w)))
        if not need_dx:
            return
        kind = _dgrad_kind(co, ci, k) if stride == 1 else "taps_t"
        if kind == "taps_t":
            add(w, lambda t, k=k, co=co, ci=ci: t.permute(2, 3, 1, 0).reshape(k * k, ci, co), ("taps_t", id(w)))
        else:
            add(w, lambda t, kind=kind, k=k, co=co, ci=ci: _pack_fn(kind, ci, co, k)(t.flip(2, 3).transpose(0, 1)),
                ("dgrad", id(w)))

    def dcn(d):
        com, w = d.conv_offset_mask, d.weight
        cout = w.shape[0]
        add(com.weight, _pack_fn("dcn", 27, 32, 3), ("fwd", id(com.weight)))
        add(w, _pack_fn("dcn", cout, 32, 3), ("fwd", id(w)))
        add(w, lambda t, cout=cout: t.reshape(cout, 32, 9).permute(2, 0, 1), ("wtaps", id(w)))
        add(com.weight, lambda t: _pack_fn("dcn", 32, 32, 3)(torch.cat([t, t.new_zeros(5, 32, 3, 3)]).flip(2, 3)
                                                                  .transpose(0, 1)), ("offdgrad", id(com.weight)))

    block(fnet.conv0[0], 3, 1, need_dx=False)
    block(fnet.conv0[1], 3, 1)
    block(fnet.conv1[0], 5, 2)
    block(fnet.conv1[1], 3, 1)
    block(fnet.conv1[2], 3, 1)
    block(fnet.conv2[0], 5, 2)
    block(fnet.conv2[1], 3, 1)
    block(fnet.conv2[2], 3, 1)
    for seq, k in ((fnet.out1, 1), (fnet.out2, 3), (fnet.out3, 3)):
        block(seq[0], k, 1, head3x3=k == 3)
        dcn(seq[1])
        dcn(seq[4])
        dcn(seq[7])
    for conv in (fnet.inner1, fnet.inner2):
        w = conv.weight
        co, ci = w.shape[0], w.shape[1]
        add(w, lambda t, co=co, ci=ci: t.permute(2, 3, 1, 0).reshape(1, ci, co), ("taps_t", id(w)))
    # a parameter appearing twice (forward and data-gradient packs) is passed twice: gather_packs keys
    # its index on the tensors' shapes, and the specs name their own tensor
    outs = gather_packs(tensors, specs, "featurenet_train")
    for key, o in zip(keys, outs):
        table[key] = o
    return table


def _taps(w):
    """Conv2d weight [Co][Ci][k][k] -> [k*k][Co][Ci] (the forward gather)."""
    co, ci, k, _ = w.shape
    return w.detach().float().permute(2, 3, 0, 1).reshape(k * k, co, ci).contiguous()


def _taps_t(w):
    """[Co][Ci][k][k] -> [k*k][Ci][Co] (the data gradient's transposed gather)."""
    co, ci, k, _ = w.shape
    return w.detach().float().permute(2, 3, 1, 0).reshape(k * k, ci, co).contiguous()


def _untaps(dw, shape):
    """[k*k][Co][Ci] -> [Co][Ci][k][k]."""
    co, ci, k, _ = shape
    return dw.reshape(k, k, co, ci).permute(2, 3, 0, 1).contiguous()


class _Tape:
    """What the forward keeps for the backward, and the BatchNorm statistics per view."""

    def __init__(self, n_views):
        self.n = n_views
        self.stats = []  # (bn module, (mean [N, C], var [N, C]) per view, pixels per view)


def _bn_relu_views(tape, z, bn):
    """relu(BatchNorm_train(z)) with statistics per view (z [N,h,w,C] NHWC): one grouped launch each
    for the statistics and the normalisation (group = view)."""
    mean, var = ops.bn_stats_grouped(z)
    y = ops.bn_relu_train_grouped(z, mean, var, bn.weight.detach(), bn.bias.detach(), bn.eps)
    tape.stats.append((bn, (mean, var), z.shape[1] * z.shape[2]))
    return y, (mean, var)


def _bn_relu_views_backward(dy, z, per, bn):
    mean, var = per
    return ops.bn_relu_backward_grouped(dy.contiguous(), z, mean, var, bn.weight.detach(), bn.bias.detach(), bn.eps)


# ------------------------------------------------------------------------- layers: forward records
def _block_fwd(tape, blk, x, k, stride, nchw_input=False, head3x3=False):
    """Conv2d (no bias) + BatchNorm (train) + ReLU (models/module.py:24-61) -> (y NHWC, record)."""
    w = blk.conv.weight
    cout = w.shape[0]
    pw = _pk(("fwd", id(w)))
    if head3x3:
        _, z = ops.conv3x3_nhwc(x, pw if pw is not None else device_pack("dcn", w), bn=None, relu=False)
    else:
        z = ops.conv2d_bn_relu(x, pw if pw is not None else device_pack("conv2d", w), cout, k, stride, bn=None,
                               relu=False, nchw_input=nchw_input)
    y, per = _bn_relu_views(tape, z, blk.bn)
    return y, ("block", blk, x, z, per, k, stride, nchw_input)


def _dcn_fwd(dcn, x, want_nchw=False):
    com = dcn.conv_offset_mask
    pwo, pw = _pk(("fwd", id(com.weight))), _pk(("fwd", id(dcn.weight)))
    u, om, out = ops.dcn_forward_train(x, pwo if pwo is not None else device_pack("dcn", com.weight),
                                       com.bias.detach().float().contiguous(),
                                       pw if pw is not None else device_pack("dcn", dcn.weight),
                                       dcn.bias.detach().float().contiguous(), dcn.cout, want_nchw=want_nchw)
    return u, om, out


def _head_fwd(tape, seq, x, first_k):
    """out{1,2,3} (models/module.py:362-395): block, DCN-BN-ReLU, DCN-BN-ReLU, DCN -> NCHW output."""
    h0, r0 = _block_fwd(tape, seq[0], x, first_k, 1, head3x3=first_k == 3)
    u1, om1, _ = _dcn_fwd(seq[1], h0)
    h1, p1 = _bn_relu_views(tape, u1, seq[2])
    u2, om2, _ = _dcn_fwd(seq[4], h1)
    h2, p2 = _bn_relu_views(tape, u2, seq[5])
    _, om3, out = _dcn_fwd(seq[7], h2, want_nchw=True)
    return out, ("head", seq, r0, (h0, om1, u1, p1), (h1, om2, u2, p2), (h2, om3))


# ------------------------------------------------------------------------- layers: backward
def _acc(grads, p, g):
    grads[id(p)] = g if id(p) not in grads else grads[id(p)] + g


def _defer(grads, p, raw, fn):
    """A weight gradient in a kernel's layout, re-laid out by fn at the end of the backward together with
    all the others (one packing.gather_packs call instead of a permute/slice launch each)."""
    if os.environ.get("TMVS_NO_STEP_PACKS") == "1":
        _acc(grads, p, fn(raw).contiguous())
        return
    grads.setdefault("__defer__", []).append((p, raw, fn))


def _flush_deferred(grads):
    pend = grads.pop("__defer__", [])
    if not pend:
        return
    outs = gather_packs([r for _, r, _ in pend], [(i, fn) for i, (_, _, fn) in enumerate(pend)], "featurenet_grads")
    for (p, _, _), o in zip(pend, outs):
        _acc(grads, p, o)


def _untaps_fn(shape):
    co, ci, k, _ = shape
    return lambda t: t.reshape(k, k, co, ci).permute(2, 3, 0, 1)


def _flip_t(w):
    """The data gradient of a stride-1 'same' conv is a forward conv of dz with the weight transposed
    (in <-> out) and flipped in both spatial axes: W'[ci][co][kh][kw] = W[co][ci][k-1-kh][k-1-kw]."""
    return w.detach().float().flip(2, 3).transpose(0, 1).contiguous()


# (dz channels, dx channels, k) that tmvs_conv2d_bn_relu takes as a forward conv (stride 1)
_MFMA_DGRAD = {(8, 8, 3), (16, 16, 3), (32, 32, 1)}


def dgrad_same(dz, w, out_hw):
    """Data gradient of Conv2d(k, stride 1, padding k//2) (models/module.py:24-61) as a forward conv on
    the MFMA inference kernels (tmvs_conv3x3_nhwc for 32 -> 32 3x3, tmvs_conv2d_bn_relu otherwise),
    falling back to the VALU transposed gather for shapes those kernels do not take."""
    co, ci, k, _ = w.shape
    kind = _dgrad_kind(co, ci, k)
    pd = _pk(("dgrad", id(w))) if kind != "taps_t" else _pk(("taps_t", id(w)))
    if kind == "dcn":
        return ops.conv3x3_nhwc(dz, pd if pd is not None else device_pack("dcn", _flip_t(w)), bn=None, relu=False)[1]
    if kind == "conv2d":
        return ops.conv2d_bn_relu(dz, pd if pd is not None else device_pack("conv2d", _flip_t(w)), ci, k, 1, bn=None,
                                  relu=False)
    return ops.conv2d_generic(dz, pd if pd is not None else _taps_t(w), ci, out_hw, k, 1, k // 2, transposed=True)


def _block_bwd(rec, dy, grads, need_dx=True):
    _, blk, x, z, per, k, stride, nchw_input = rec
    dz, dg, db = _bn_relu_views_backward(dy, z, per, blk.bn)
    _acc(grads, blk.bn.weight, dg)
    _acc(grads, blk.bn.bias, db)
    w = blk.conv.weight
    pad = k // 2
    xg = x.permute(0, 2, 3, 1).contiguous() if nchw_input else x
    _defer(grads, w, ops.conv2d_wgrad(dz, xg, k, stride, pad), _untaps_fn(w.shape))
    if not need_dx:
        return None
    if stride == 1:
        return dgrad_same(dz, w, (xg.shape[1], xg.shape[2]))
    pt = _pk(("taps_t", id(w)))
    return ops.conv2d_generic(dz, pt if pt is not None else _taps_t(w), w.shape[1], (xg.shape[1], xg.shape[2]), k,
                              stride, pad, transposed=True)


def _dcn_bwd(dcn, x, om, dy, grads):
    """DCN.forward's backward: (dcol, d offsets / mask logits, dW, dx scatter) then the offset/mask
    conv (3x3, 32 -> 27, bias). Returns dx [N,h,w,32]."""
    w = dcn.weight
    cout = w.shape[0]
    w_taps = _pk(("wtaps", id(w)))
    if w_taps is None:
        w_taps = w.detach().float().reshape(cout, 32, 9).permute(2, 0, 1).contiguous()
    dx, dom, dw = ops.dcn_backward_set(x, om, w_taps, dy)  # dx written: no zero fill per call
    _defer(grads, w, dw, lambda t, cout=cout: t.permute(1, 2, 0).reshape(cout, 32, 3, 3))
    _acc(grads, dcn.bias, ops.colsum(dy))
    # the offset/mask conv (3x3, 32 -> 27, bias) on dom padded to 32 channels (27..31 zero): its
    # weight gradient rows 27..31 are dropped, its data gradient reads them against zero weights
    com = dcn.conv_offset_mask
    _defer(grads, com.weight, ops.conv2d_wgrad(dom, x, 3, 1, 1),
           lambda t: t[:, :27].reshape(3, 3, 27, 32).permute(2, 3, 0, 1))
    _defer(grads, com.bias, ops.colsum(dom), lambda t: t[:27])
    # dx += its data gradient (dgrad_same's 32 -> 32 3x3 form on the weight padded to 32 output rows,
    # packed by one gather), added in the conv's epilogue
    po = _pk(("offdgrad", id(com.weight)))
    ops.conv3x3_nhwc_acc(dom, po if po is not None else offset_dgrad_pack(com.weight), dx)
    return dx


def _head_bwd(rec, dout_nchw, grads):
    _, seq, r0, (h0, om1, u1, p1), (h1, om2, u2, p2), (h2, om3) = rec
    dy3 = dout_nchw.permute(0, 2, 3, 1).contiguous()
    dh2 = _dcn_bwd(seq[7], h2, om3, dy3, grads)
    du2, dg, db = _bn_relu_views_backward(dh2, u2, p2, seq[5])
    _acc(grads, seq[5].weight, dg)
    _acc(grads, seq[5].bias, db)
    dh1 = _dcn_bwd(seq[4], h1, om2, du2, grads)
    du1, dg, db = _bn_relu_views_backward(dh1, u1, p1, seq[2])
    _acc(grads, seq[2].weight, dg)
    _acc(grads, seq[2].bias, db)
    dh0 = _dcn_bwd(seq[1], h0, om1, du1, grads)
    return _block_bwd(r0, dh0, grads)


def _inner_bwd(conv, d, lat, grads):
    """inner{1,2} = Conv2d(cl, 32, 1, bias) of the FPN merge: grads, and d lat [N,h,w,cl]."""
    w = conv.weight
    _defer(grads, w, ops.conv2d_wgrad(d, lat, 1, 1, 0), _untaps_fn(w.shape))
    _acc(grads, conv.bias, ops.colsum(d))
    pt = _pk(("taps_t", id(w)))
    return ops.conv2d_generic(d, pt if pt is not None else _taps_t(w), w.shape[1], (lat.shape[1], lat.shape[2]), 1, 1, 0)


class _FeatureNetTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, imgs, fnet, tape, *params):
        ctx.packs = _prepare_packs(fnet)
        x = imgs.float().contiguous()
        c00, r00 = _block_fwd(tape, fnet.conv0[0], x, 3, 1, nchw_input=True)
        conv0, r01 = _block_fwd(tape, fnet.conv0[1], c00, 3, 1)
        c10, r10 = _block_fwd(tape, fnet.conv1[0], conv0, 5, 2)
        c11, r11 = _block_fwd(tape, fnet.conv1[1], c10, 3, 1)
        conv1, r12 = _block_fwd(tape, fnet.conv1[2], c11, 3, 1)
        c20, r20 = _block_fwd(tape, fnet.conv2[0], conv1, 5, 2)
        c21, r21 = _block_fwd(tape, fnet.conv2[1], c20, 3, 1)
        conv2, r22 = _block_fwd(tape, fnet.conv2[2], c21, 3, 1)
        s1, h1 = _head_fwd(tape, fnet.out1, conv2, 1)
        intra1 = ops.fpn_merge(conv2, conv1, *fnet._inner(fnet.inner1, conv2.device))
        s2, h2 = _head_fwd(tape, fnet.out2, intra1, 3)
        intra2 = ops.fpn_merge(intra1, conv0, *fnet._inner(fnet.inner2, conv2.device))
        s3, h3 = _head_fwd(tape, fnet.out3, intra2, 3)
        ctx.recs = (r00, r01, r10, r11, r12, r20, r21, r22, h1, h2, h3)
        ctx.lat = (conv0, conv1)
        ctx.fnet = fnet
        ctx.param_ids = [id(p) for p in params]
        return s1, s2, s3

    @staticmethod
    def backward(ctx, d1, d2, d3):
        with _active_packs(ctx.packs):  # this forward's packs, not the most recent forward's
            return _FeatureNetTrain._backward(ctx, d1, d2, d3)

    @staticmethod
    def _backward(ctx, d1, d2, d3):
        r00, r01, r10, r11, r12, r20, r21, r22, h1, h2, h3 = ctx.recs
        conv0, conv1 = ctx.lat
        fnet = ctx.fnet
        grads = {}
        # out3 head on intra2 = up2(intra1) + inner2(conv0)
        dconv0 = dintra1 = None
        if d3 is not None:
            dintra2 = _head_bwd(h3, d3, grads)
            dintra1 = ops.nearest_up2_backward_nhwc(dintra2)
            dconv0 = _inner_bwd(fnet.inner2, dintra2, conv0, grads)
        # out2 head on intra1 = up2(conv2) + inner1(conv1)
        if d2 is not None:
            dh = _head_bwd(h2, d2, grads)
            dintra1 = dh if dintra1 is None else dintra1.add_(dh)
        dconv2 = dconv1 = None
        if dintra1 is not None:
            dconv2 = ops.nearest_up2_backward_nhwc(dintra1)
            dconv1 = _inner_bwd(fnet.inner1, dintra1, conv1, grads)
        if d1 is not None:
            dh = _head_bwd(h1, d1, grads)
            dconv2 = dh if dconv2 is None else dconv2.add_(dh)
        # trunk, in reverse; gradients meeting at conv1 / conv0 are summed
        if dconv2 is None:
            dconv2 = torch.zeros_like(r22[3])
        d = _block_bwd(r22, dconv2, grads)
        d = _block_bwd(r21, d, grads)
        d = _block_bwd(r20, d, grads)
        d = d if dconv1 is None else d.add_(dconv1)
        d = _block_bwd(r12, d, grads)
        d = _block_bwd(r11, d, grads)
        d = _block_bwd(r10, d, grads)
        d = d if dconv0 is None else d.add_(dconv0)
        d = _block_bwd(r01, d, grads)
        _block_bwd(r00, d, grads, need_dx=False)
        _flush_deferred(grads)
        return (None, None, None, *[grads.get(i) for i in ctx.param_ids])


def featurenet_train(fnet, imgs):
    """FeatureNet.forward in train mode for one sample's views imgs [N,3,H,W] -> (stage1, stage2, stage3)
    NCHW, differentiable w.r.t. fnet's parameters; updates the BatchNorm running statistics per view
    as the reference's per-view calls do."""
    if not imgs.is_cuda:
        raise RuntimeError("featurenet_train runs on the GPU only (no CPU fallback)")
    if imgs.dim() != 4 or imgs.shape[1] != 3:
        raise ValueError("featurenet_train: imgs must be [N, 3, H, W] (one sample's views)")
    tape = _Tape(imgs.shape[0])
    params = list(fnet.parameters())
    with torch.cuda.device(imgs.device):
        s1, s2, s3 = _FeatureNetTrain.apply(imgs, fnet, tape, *params)
        # views in order, as the reference's per-view calls (closed form, bn_running.py)
        update_running_stats([(bn, mean, var, n) for bn, (mean, var), n in tape.stats], BN_MOMENTUM)
    return s1, s2, s3
