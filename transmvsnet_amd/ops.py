"""Torch-tensor wrappers over the C-ABI (device memory + current HIP stream in, status checked).

Each op mirrors one reference callable (file:line in include/transmvs.h). Tensors must be
fp32, contiguous and on the GPU; nothing here computes on the CPU except the 4x4 camera
algebra that produces kernel arguments (proj_rows), which is done exactly as the
reference does it so the warp coordinates match bit for bit.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

_lib_h = _lib.load


_TIMER = None


def set_timer(timer):
    """Install an object with begin(name) -> token / end(token) around every C-ABI launch
    (bench.py uses HIP events on the launching stream); None disables."""
    global _TIMER
    _TIMER = timer


class _Span:
    __slots__ = ("tok",)

    def __init__(self, name):
        self.tok = _TIMER.begin(name) if _TIMER is not None else None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        if self.tok is not None:
            _TIMER.end(self.tok)


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _stream():
    """The current HIP stream of the current device. Every public op below runs under a device guard
    set from its first GPU tensor argument (_on_tensor_device), so this is that tensor's device."""
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _on_tensor_device(fn):
    """Run `fn` with the current device = the device of its first GPU tensor argument, so its kernels
    launch on that device and on that device's current stream (a model on cuda:1 works without
    torch.cuda.set_device(1))."""
    import functools

    @functools.wraps(fn)
    def wrapped(*args, **kwargs):
        for a in (*args, *kwargs.values()):
            if isinstance(a, torch.Tensor) and a.is_cuda:
                if a.device.index == torch.cuda.current_device():
                    return fn(*args, **kwargs)
                with torch.cuda.device(a.device):
                    return fn(*args, **kwargs)
        return fn(*args, **kwargs)
    wrapped.device_guarded = True
    return wrapped


def _dev(t, name):
    if t is None:
        return
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a GPU tensor (the HIP path has no CPU fallback)")
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous float32")


# ----------------------------------------------------------------- host-side parameter math
def bn_fold(gamma, beta, mean, var, eps=1e-5):
    """(alpha, shift) CPU float32 arrays, reference batch_norm eval semantics (tmvs_bn_fold)."""
    g = np.ascontiguousarray(gamma.detach().cpu().numpy(), np.float32)
    b = np.ascontiguousarray(beta.detach().cpu().numpy(), np.float32)
    m = np.ascontiguousarray(mean.detach().cpu().numpy(), np.float32)
    v = np.ascontiguousarray(var.detach().cpu().numpy(), np.float32)
    a = np.empty_like(g)
    s = np.empty_like(g)
    with _Span("tmvs_bn_fold"):
        _lib.check(_lib_h().tmvs_bn_fold(g.ctypes.data, b.ctypes.data, m.ctypes.data, v.ctypes.data, g.size,
                                         ctypes.c_float(eps), a.ctypes.data, s.ctypes.data), "tmvs_bn_fold")
    return a, s


def compose_proj(proj):
    """[B,2,4,4] -> [B,4,4] with rows 0..2 = K·E[:3,:4] (models/TransMVSNet.py:75-78), CPU fp32."""
    new = proj[:, 0].clone()
    new[:, :3, :4] = torch.matmul(proj[:, 1, :3, :3], proj[:, 0, :3, :4])
    return new


def proj_rows(proj_matrix_stage):
    """[B,N,2,4,4] -> float32 [B, N-1, 12] = rows of P_src·P_ref^-1 (models/module.py:295-297).

    Same torch-CPU fp32 ops as the reference, so the homography is bit-identical.
    """
    pm = proj_matrix_stage.detach().to("cpu", torch.float32)
    ref = compose_proj(pm[:, 0])
    inv = torch.inverse(ref)
    rows = []
    for v in range(1, pm.shape[1]):
        p = torch.matmul(compose_proj(pm[:, v]), inv)
        rows.append(p[:, :3, :4].reshape(pm.shape[0], 12))
    return torch.stack(rows, 1).contiguous().numpy()


_ROT_ORDER = {}


def host_rot_order(n_pixels):
    """'fma' or 'plain': how THIS host's torch.matmul rounds homo_warping's rot·(x, y, 1)
    (models/module.py:303, a [3,3] x [3,H*W] bmm). The reference's sample coordinates depend on it:
    MKL contracts the 3-term dot into fmaf(r1, y, r0·x) + r2 on AVX-512 Xeons and computes
    (r0·x + r1·y) + r2 on AMD EPYC (scripts/diag/warp_bits.py). Probed once per size with the
    reference's own call shape; the warp kernels then reproduce the host's coordinates bit for bit."""
    order = _ROT_ORDER.get(n_pixels)
    if order is None:
        g = np.random.default_rng(12345)
        w = 1 << max(1, int(np.ceil(np.log2(max(2.0, np.sqrt(n_pixels))))))
        xs = (np.arange(n_pixels) % w).astype(np.float32)
        ys = (np.arange(n_pixels) // w).astype(np.float32)
        rot = g.uniform(-1.0, 1.0, (3, 3)).astype(np.float32)
        rot[:, 2] *= 300.0
        xyz = torch.from_numpy(np.stack([xs, ys, np.ones_like(xs)]))[None]
        got = torch.matmul(torch.from_numpy(rot)[None], xyz)[0].numpy()
        r0, r1, r2 = rot[:, 0:1], rot[:, 1:2], rot[:, 2:3]
        fma = (r1.astype(np.float64) * ys + (r0 * xs)).astype(np.float32) + r2
        plain = (r0 * xs + r1 * ys) + r2
        order = "plain" if (plain == got).sum() > (fma == got).sum() else "fma"
        _ROT_ORDER[n_pixels] = order
    return order


def warp_flags(rot_order, n_pixels):
    """TMVS_WARP_ROT_PLAIN or 0 for rot_order 'fma' / 'plain' / 'auto' (= host_rot_order)."""
    if rot_order == "auto":
        rot_order = host_rot_order(n_pixels)
    if rot_order not in ("fma", "plain"):
        raise ValueError(f"rot_order must be 'auto', 'fma' or 'plain', got {rot_order!r}")
    return _lib.WARP_ROT_PLAIN if rot_order == "plain" else 0


# ----------------------------------------------------------------- ops
def stage_hypotheses(depth_values, prev_depth, ndepth, ratio, full_hw, stage_scale):
    """Stage glue (models/TransMVSNet.py:174-204): -> [B, D, H/s, W/s]."""
    _dev(depth_values, "depth_values")
    _dev(prev_depth, "prev_depth")
    b = depth_values.shape[0]
    h, w = full_hw
    out = torch.empty(b, ndepth, h // stage_scale, w // stage_scale, device=depth_values.device)
    ph, pw = (prev_depth.shape[1], prev_depth.shape[2]) if prev_depth is not None else (0, 0)
    with _Span("tmvs_stage_hypotheses"):
        _lib.check(_lib_h().tmvs_stage_hypotheses(_ptr(depth_values), depth_values.shape[1], _ptr(prev_depth), ph, pw, b,
                                                  ndepth, ctypes.c_float(ratio), h, w, stage_scale, _ptr(out), _stream()),
                   "tmvs_stage_hypotheses")
    return out


def warp_corr(ref_nhwc, src_nhwc, proj12, hyp, view_w_in=None, vw_shift=0, vw_offset=0, vw_total=None,
              pw_params=None, partial=False, view_w_out=None, sim_out=None, wsum_out=None, rot_order="auto"):
    """Fused cost volume (models/TransMVSNet.py:58-93). ref [B,H,W,C], src [B,V,H,W,C], proj12 HOST [B,V,12].

    Returns sim [B,D,H,W] (and w_sum [B,H,W] when partial) ; stage 1 writes view_w_out [B,vw_total,H,W].
    rot_order: the reference's rounding of rot·(x, y, 1) ('auto' = this host's torch, host_rot_order).
    """
    for t, n in ((ref_nhwc, "ref"), (src_nhwc, "src"), (hyp, "hyp"), (view_w_in, "view_w_in"), (view_w_out, "view_w_out")):
        _dev(t, n)
    b, v, h, w, c = src_nhwc.shape
    d = hyp.shape[1]
    vw_total = v if vw_total is None else vw_total
    proj = np.ascontiguousarray(proj12, np.float32).reshape(b, v, 12)
    sim = torch.empty(b, d, h, w, device=hyp.device) if sim_out is None else sim_out
    wsum = (torch.empty(b, h, w, device=hyp.device) if wsum_out is None else wsum_out) if partial else None
    if sim.shape != (b, d, h, w) or not sim.is_contiguous():
        raise ValueError(f"sim_out must be a contiguous [{b},{d},{h},{w}] tensor")
    if wsum is not None and (wsum.numel() != b * h * w or not wsum.is_contiguous()):
        raise ValueError(f"wsum_out must be a contiguous [{b},{h},{w}] tensor")
    if view_w_in is None:
        if view_w_out is None:
            view_w_out = torch.empty(b, vw_total, h, w, device=hyp.device)
        pw = np.ascontiguousarray(pw_params, np.float32)
        assert pw.size == _lib.PW_NPARAMS
        pw_ptr = pw.ctypes.data
    else:
        pw_ptr = None
    with _Span("tmvs_warp_corr"):
        _lib.check(_lib_h().tmvs_warp_corr(_ptr(ref_nhwc), _ptr(src_nhwc), proj.ctypes.data, _ptr(hyp), _ptr(view_w_in),
                                           vw_shift, vw_offset, vw_total, pw_ptr, b, v, c, d, h, w,
                                           (_lib.WARP_PARTIAL if partial else 0) | warp_flags(rot_order, h * w),
                                           _ptr(sim), _ptr(wsum),
                                           _ptr(view_w_out if view_w_in is None else None), _stream()), "tmvs_warp_corr")
    return sim, wsum, (view_w_out if view_w_in is None else None)


def aggregate_finalize(sim_sum, w_sum):
    _dev(sim_sum, "sim_sum")
    _dev(w_sum, "w_sum")
    b, d, h, w = sim_sum.shape
    with _Span("tmvs_aggregate_finalize"):
        _lib.check(_lib_h().tmvs_aggregate_finalize(_ptr(sim_sum), _ptr(w_sum), b, d, h, w, _stream()),
                   "tmvs_aggregate_finalize")
    return sim_sum


def homo_warping(src_fea, src_proj, ref_proj, depth_values, rot_order="auto"):
    """Seam-compatible homo_warping (models/module.py:284-322): [B,C,H,W] -> [B,C,D,H,W]."""
    _dev(src_fea, "src_fea")
    _dev(depth_values, "depth_values")
    b, c, h, w = src_fea.shape
    d = depth_values.shape[1]
    p = torch.matmul(src_proj.detach().cpu().float(), torch.inverse(ref_proj.detach().cpu().float()))
    rows = np.ascontiguousarray(p[:, :3, :4].reshape(b, 12).numpy(), np.float32)
    out = torch.empty(b, c, d, h, w, device=src_fea.device)
    with _Span("tmvs_homo_warping"):
        _lib.check(_lib_h().tmvs_homo_warping(_ptr(src_fea), rows.ctypes.data, _ptr(depth_values.contiguous()), b, c, d,
                                              h, w, warp_flags(rot_order, h * w), _ptr(out), _stream()),
                   "tmvs_homo_warping")
    return out


def softmax_wta(logits, hyp, clamp=(425.0, 935.0)):
    """prob, depth (clamped), depth_raw, conf (models/TransMVSNet.py:97-103,217-221)."""
    _dev(logits, "logits")
    _dev(hyp, "hyp")
    b, d, h, w = logits.shape
    prob = torch.empty_like(logits)
    depth = torch.empty(b, h, w, device=logits.device)
    raw = torch.empty_like(depth)
    conf = torch.empty_like(depth)
    with _Span("tmvs_softmax_wta"):
        _lib.check(_lib_h().tmvs_softmax_wta(_ptr(logits), _ptr(hyp), b, d, h, w, ctypes.c_float(clamp[0]),
                                             ctypes.c_float(clamp[1]), _ptr(prob), _ptr(depth), _ptr(raw), _ptr(conf),
                                             _stream()), "tmvs_softmax_wta")
    return prob, depth, raw, conf


def costregnet(x, weights: "_lib.CostRegWeights", keepalive=None):
    """CostRegNet forward (models/module.py:447-456): [B,D,H,W] -> logits [B,D,H,W]."""
    _dev(x, "x")
    b, d, h, w = x.shape
    nbytes = _lib_h().tmvs_costregnet_workspace(b, d, h, w, weights.base_ch)
    ws = torch.empty(nbytes // 4 + 64, device=x.device)
    out = torch.empty_like(x)
    with _Span("tmvs_costregnet"):
        _lib.check(_lib_h().tmvs_costregnet(_ptr(x), b, d, h, w, ctypes.byref(weights), _ptr(ws), ws.numel() * 4,
                                            _ptr(out), _stream()), "tmvs_costregnet")
    return out


def costregnet_wta(x, weights: "_lib.CostRegWeights", hyp, clamp=(425.0, 935.0)):
    """CostRegNet -> softmax/WTA (models/module.py:447-456, TransMVSNet.py:97-103,214-221) in one
    call: prob, depth (clamped), depth_raw, conf, equal bit for bit to costregnet -> softmax_wta."""
    _dev(x, "x")
    _dev(hyp, "hyp")
    b, d, h, w = x.shape
    if tuple(hyp.shape) != (b, d, h, w):
        raise ValueError(f"costregnet_wta: hyp shape {tuple(hyp.shape)} != volume shape {(b, d, h, w)}")
    nbytes = _lib_h().tmvs_costregnet_workspace(b, d, h, w, weights.base_ch)
    ws = torch.empty(nbytes // 4 + 64, device=x.device)
    prob = torch.empty_like(x)
    depth = torch.empty(b, h, w, device=x.device)
    raw = torch.empty_like(depth)
    conf = torch.empty_like(depth)
    with _Span("tmvs_costregnet"):
        _lib.check(_lib_h().tmvs_costregnet_wta(_ptr(x), _ptr(hyp), b, d, h, w, ctypes.byref(weights), _ptr(ws),
                                                ws.numel() * 4, ctypes.c_float(clamp[0]), ctypes.c_float(clamp[1]),
                                                _ptr(prob), _ptr(depth), _ptr(raw), _ptr(conf), _stream()),
                   "tmvs_costregnet_wta")
    return prob, depth, raw, conf


def conv3d_bn_relu(x, wpk, alpha, shift, cout, stride):
    b, d, h, w, cin = x.shape
    do, ho, wo = ((d - 1) // 2 + 1, (h - 1) // 2 + 1, (w - 1) // 2 + 1) if stride == 2 else (d, h, w)
    y = torch.empty(b, do, ho, wo, cout, device=x.device)
    with _Span("tmvs_conv3d_bn_relu"):
        _lib.check(_lib_h().tmvs_conv3d_bn_relu(_ptr(x), b, cin, d, h, w, _ptr(wpk), _ptr(alpha), _ptr(shift), cout,
                                                stride, _ptr(y), _stream()), "tmvs_conv3d_bn_relu")
    return y


def deconv3d_bn_relu_add(x, wpk, alpha, shift, cout, skip):
    b, d, h, w, cin = x.shape
    y = torch.empty(b, 2 * d, 2 * h, 2 * w, cout, device=x.device)
    with _Span("tmvs_deconv3d_bn_relu_add"):
        _lib.check(_lib_h().tmvs_deconv3d_bn_relu_add(_ptr(x), b, cin, d, h, w, _ptr(wpk), _ptr(alpha), _ptr(shift),
                                                      cout, _ptr(skip), _ptr(y), _stream()), "tmvs_deconv3d_bn_relu_add")
    return y


def fmt_embed(feat_nchw, pe, out_tokens):
    """x + PE, 'n c h w -> n (h w) c' (FMT.py:152): feat [nv,C,H,W] -> tokens [nv,H*W,C] (written in place)."""
    nv, c, h, w = feat_nchw.shape
    with _Span("tmvs_fmt_embed"):
        _lib.check(_lib_h().tmvs_fmt_embed(_ptr(feat_nchw), c * h * w, _ptr(pe), pe.shape[1], pe.shape[2], nv, c, h, w,
                                           _ptr(out_tokens), _stream()), "tmvs_fmt_embed")
    return out_tokens


def fmt_kv(source_tokens, enc_w, out=None):
    """(KV, Ksum) of one encoder layer over source tokens [nv,S,32] -> [nv,160]."""
    nv, s, _ = source_tokens.shape
    nbytes = _lib_h().tmvs_fmt_kv_workspace(nv, s)
    ws = torch.empty(max(1, nbytes // 4), device=source_tokens.device)
    kv = out if out is not None else torch.empty(nv, _lib.KV_NFLOATS, device=source_tokens.device)
    with _Span("tmvs_fmt_kv"):
        _lib.check(_lib_h().tmvs_fmt_kv(_ptr(source_tokens), nv, s, _ptr(enc_w), _ptr(ws), ws.numel() * 4, _ptr(kv),
                                        _stream()), "tmvs_fmt_kv")
    return kv


def fmt_apply(x_tokens, kv, enc_w, shared_kv=False):
    """Rest of EncoderLayer.forward in place on x [nv,L,32] (FMT.py:96-111)."""
    nv, l, _ = x_tokens.shape
    with _Span("tmvs_fmt_apply"):
        _lib.check(_lib_h().tmvs_fmt_apply(_ptr(x_tokens), nv, l, _ptr(kv), 0 if shared_kv else _lib.KV_NFLOATS,
                                           _ptr(enc_w), _stream()), "tmvs_fmt_apply")
    return x_tokens


def fmt_pathway(coarse_nhwc, lateral_nchw, w_reduce, w_smooth, out=None):
    """smooth(up2(reduce(coarse)) + lateral) (FMT.py:221-228): coarse [nv,h,w,cc], lateral [nv,cf,2h,2w].

    out: optional contiguous [nv,2h,2w,cf] destination (e.g. a view slice of a larger batch)."""
    nv, h, w, cc = coarse_nhwc.shape
    cf = lateral_nchw.shape[1]
    if out is None:
        out = torch.empty(nv, 2 * h, 2 * w, cf, device=coarse_nhwc.device)
    elif tuple(out.shape) != (nv, 2 * h, 2 * w, cf) or not out.is_contiguous():
        raise ValueError(f"fmt_pathway: out must be a contiguous [{nv},{2 * h},{2 * w},{cf}] tensor")
    with _Span("tmvs_fmt_pathway"):
        _lib.check(_lib_h().tmvs_fmt_pathway(_ptr(coarse_nhwc), _ptr(lateral_nchw), cf * 4 * h * w, _ptr(w_reduce),
                                             _ptr(w_smooth), nv, cc, cf, h, w, _ptr(out), _stream()), "tmvs_fmt_pathway")
    return out


# ----------------------------------------------------------------- native orchestration
def fmt_forward(stage1_nchw, pe, enc_list, tokens=None, side_stream=None):
    """Whole FMT (models/FMT.py:147-177): stage1 [nv,32,H,W] -> tokens [nv,H*W,32].

    side_stream (a torch.cuda.Stream): the reference view's chain runs on it, concurrently with the source
    views (tmvs_fmt_forward_split; bitwise the same tokens). It forks from and joins back into the current
    stream inside the call.
    """
    _dev(stage1_nchw, "stage1")
    nv, c, h, w = stage1_nchw.shape
    tokens = torch.empty(nv, h * w, c, device=stage1_nchw.device) if tokens is None else tokens
    split = side_stream is not None and nv > 1
    lib = _lib_h()
    nbytes = lib.tmvs_fmt_forward_split_workspace(nv, h * w) if split else lib.tmvs_fmt_forward_workspace(nv, h * w)
    ws = torch.empty(nbytes // 4 + 64, device=stage1_nchw.device)
    ptrs = (ctypes.c_void_p * 8)(*[e.data_ptr() for e in enc_list])
    args = (_ptr(stage1_nchw), c * h * w, _ptr(pe), pe.shape[1], pe.shape[2], nv, h, w, ptrs, _ptr(ws), ws.numel() * 4,
            _ptr(tokens), _stream())
    with _Span("tmvs_fmt_forward"):
        if split:
            _lib.check(lib.tmvs_fmt_forward_split(*args, side_stream.cuda_stream), "tmvs_fmt_forward_split")
            if not torch.cuda.is_current_stream_capturing():  # allocator: ws / tokens are also used on the side stream
                ws.record_stream(side_stream)
                tokens.record_stream(side_stream)
        else:
            _lib.check(lib.tmvs_fmt_forward(*args), "tmvs_fmt_forward")
    return tokens


def depth_stage(depth_values, prev_depth, feat_nhwc, ndepth, ratio, full_hw, stage_scale, proj12, pw_params,
                view_w, vw_shift, cr_weights, clamp=(425.0, 935.0), rot_order="auto"):
    """One cascade stage for one sample (models/TransMVSNet.py:174-221). feat [N,h,w,C] NHWC.

    Returns dict(depth, photo_confidence, prob_volume, depth_values) with a batch dim of 1, and depth_raw.
    """
    _dev(depth_values, "depth_values")
    _dev(prev_depth, "prev_depth")
    _dev(feat_nhwc, "feat")
    _dev(view_w, "view_w")
    n, h, w, c = feat_nhwc.shape
    dev = feat_nhwc.device
    hyp = torch.empty(1, ndepth, h, w, device=dev)
    prob = torch.empty_like(hyp)
    depth = torch.empty(1, h, w, device=dev)
    raw = torch.empty_like(depth)
    conf = torch.empty_like(depth)
    nbytes = _lib_h().tmvs_depth_stage_workspace(ndepth, h, w, cr_weights.base_ch)
    ws = torch.empty(nbytes // 4 + 64, device=dev)
    proj = np.ascontiguousarray(proj12, np.float32).reshape(n - 1, 12)
    pw = None if pw_params is None else np.ascontiguousarray(pw_params, np.float32)
    ph, pwd = (prev_depth.shape[-2], prev_depth.shape[-1]) if prev_depth is not None else (0, 0)
    with _Span("tmvs_depth_stage"):
        _lib.check(_lib_h().tmvs_depth_stage(_ptr(depth_values), depth_values.shape[-1], _ptr(prev_depth), ph, pwd,
                                             _ptr(feat_nhwc), n, c, ndepth, ctypes.c_float(ratio), full_hw[0], full_hw[1],
                                             stage_scale, proj.ctypes.data, None if pw is None else pw.ctypes.data,
                                             _ptr(view_w), vw_shift, warp_flags(rot_order, h * w), ctypes.byref(cr_weights), _ptr(ws), ws.numel() * 4,
                                             ctypes.c_float(clamp[0]), ctypes.c_float(clamp[1]), _ptr(hyp), _ptr(prob),
                                             _ptr(depth), _ptr(raw), _ptr(conf), _stream()), "tmvs_depth_stage")
    return {"depth": depth, "photo_confidence": conf, "prob_volume": prob, "depth_values": hyp}, raw


def deform_conv2d_pack(weight):
    """HOST packing of a DCN weight [Co][32][3][3] (Co 8/16/32, or 27 for conv_offset_mask) into the
    kernel's A-fragment order (CPU float32)."""
    w = np.ascontiguousarray(weight.detach().float().cpu().numpy(), np.float32)
    co, ci = w.shape[:2]
    out = np.empty(_lib_h().tmvs_deform_conv2d_packed_floats(co), np.float32)
    _lib.check(_lib_h().tmvs_deform_conv2d_pack(w.ctypes.data, co, ci, out.ctypes.data), "tmvs_deform_conv2d_pack")
    return torch.from_numpy(out)


def deform_conv2d(x_nhwc, offset_mask, w_packed, bias, cout, bn=None, relu=False, want_nhwc=False):
    """DCN.forward's deform_conv2d (models/dcn.py:71-80) + optional folded BN / ReLU of the head.

    x_nhwc [B,H,W,32], offset_mask [B,27,H,W] (conv_offset_mask output), w_packed from
    deform_conv2d_pack (on the device). Returns out [B,cout,H,W] (and [B,H,W,cout] if want_nhwc).
    """
    for t, n in ((x_nhwc, "x_nhwc"), (offset_mask, "offset_mask"), (w_packed, "w_packed"), (bias, "bias")):
        _dev(t, n)
    b, h, w, cin = x_nhwc.shape
    if offset_mask.shape != (b, 27, h, w) or not offset_mask.is_contiguous() or not x_nhwc.is_contiguous():
        raise ValueError("deform_conv2d: expects contiguous x_nhwc [B,H,W,C] and offset_mask [B,27,H,W]")
    out = torch.empty(b, cout, h, w, device=x_nhwc.device)
    out_nhwc = torch.empty(b, h, w, cout, device=x_nhwc.device) if want_nhwc else None
    alpha, shift = bn if bn is not None else (None, None)
    with _Span("tmvs_deform_conv2d"):
        _lib.check(_lib_h().tmvs_deform_conv2d(_ptr(x_nhwc), _ptr(offset_mask), _ptr(w_packed), _ptr(bias),
                                               _ptr(alpha), _ptr(shift), int(relu), b, cin, cout, h, w, _ptr(out),
                                               _ptr(out_nhwc), _stream()), "tmvs_deform_conv2d")
    return (out, out_nhwc) if want_nhwc else out


def dcn_fused(x_nhwc, wom_packed, bom, w_packed, bias, cout, bn=None, relu=False, want_nchw=True, want_nhwc=False):
    """The whole DCN.forward (models/dcn.py:66-80): conv_offset_mask computed in-kernel, then the
    modulated deformable conv + optional folded BN / ReLU. x_nhwc [B,H,W,32] -> out [B,cout,H,W]
    and/or [B,H,W,cout] (returned as (out_nchw, out_nhwc), None where not requested)."""
    for t, n in ((x_nhwc, "x_nhwc"), (wom_packed, "wom_packed"), (bom, "bom"), (w_packed, "w_packed"), (bias, "bias")):
        _dev(t, n)
    if not (want_nchw or want_nhwc):
        raise ValueError("dcn_fused: request at least one output layout")
    b, h, w, cin = x_nhwc.shape
    if not x_nhwc.is_contiguous():
        raise ValueError("dcn_fused: expects a contiguous x_nhwc [B,H,W,C]")
    out = torch.empty(b, cout, h, w, device=x_nhwc.device) if want_nchw else None
    out_nhwc = torch.empty(b, h, w, cout, device=x_nhwc.device) if want_nhwc else None
    alpha, shift = bn if bn is not None else (None, None)
    with _Span("tmvs_dcn_fused"):
        _lib.check(_lib_h().tmvs_dcn_fused(_ptr(x_nhwc), _ptr(wom_packed), _ptr(bom), _ptr(w_packed), _ptr(bias),
                                           _ptr(alpha), _ptr(shift), int(relu), b, cin, cout, h, w, _ptr(out),
                                           _ptr(out_nhwc), _stream()), "tmvs_dcn_fused")
    return out, out_nhwc


def conv3x3_nhwc(x_nhwc, w_packed, bn=None, relu=False, bias=None, want_nchw=False, want_nhwc=True):
    """Conv2d(32, 32, 3, 1, 1) [+ bias] + folded BN + ReLU on x_nhwc [B,H,W,32] (models/module.py:24-61).
    Returns (out_nchw, out_nhwc), None where not requested."""
    for t, n in ((x_nhwc, "x_nhwc"), (w_packed, "w_packed")):
        _dev(t, n)
    if not x_nhwc.is_contiguous():
        raise ValueError("conv3x3_nhwc: expects a contiguous x_nhwc [B,H,W,32]")
    b, h, w, cin = x_nhwc.shape
    out = torch.empty(b, 32, h, w, device=x_nhwc.device) if want_nchw else None
    out_nhwc = torch.empty(b, h, w, 32, device=x_nhwc.device) if want_nhwc else None
    alpha, shift = bn if bn is not None else (None, None)
    with _Span("tmvs_conv3x3_nhwc"):
        _lib.check(_lib_h().tmvs_conv3x3_nhwc(_ptr(x_nhwc), _ptr(w_packed), _ptr(bias), _ptr(alpha), _ptr(shift),
                                              int(relu), b, cin, 32, h, w, _ptr(out), _ptr(out_nhwc), _stream()),
                   "tmvs_conv3x3_nhwc")
    return out, out_nhwc


def conv3x3_nhwc_acc(x_nhwc, w_packed, out_nhwc):
    """out_nhwc [B,H,W,32] += Conv2d(32, 32, 3, 1, 1, bias=False)(x_nhwc) in the conv's epilogue
    (tmvs_conv3x3_nhwc_acc; each element out + conv, as out.add_(conv))."""
    for t, n in ((x_nhwc, "x_nhwc"), (w_packed, "w_packed"), (out_nhwc, "out_nhwc")):
        _dev(t, n)
    if not x_nhwc.is_contiguous() or not out_nhwc.is_contiguous() or out_nhwc.shape != x_nhwc.shape:
        raise ValueError("conv3x3_nhwc_acc: expects contiguous x_nhwc and out_nhwc [B,H,W,32] of one shape")
    b, h, w, cin = x_nhwc.shape
    with _Span("tmvs_conv3x3_nhwc_acc"):
        _lib.check(_lib_h().tmvs_conv3x3_nhwc_acc(_ptr(x_nhwc), _ptr(w_packed), b, cin, 32, h, w, _ptr(out_nhwc),
                                                  _stream()), "tmvs_conv3x3_nhwc_acc")
    return out_nhwc


def fpn_merge(prev_nhwc, lat_nhwc, w_inner, b_inner):
    """interpolate(prev, 2, nearest) + Conv2d_1x1(lat) (models/module.py:409-417), all NHWC:
    prev [B,h,w,32], lat [B,2h,2w,cl] (cl 8/16), w_inner [32,cl] -> [B,2h,2w,32]."""
    for t, n in ((prev_nhwc, "prev_nhwc"), (lat_nhwc, "lat_nhwc"), (w_inner, "w_inner"), (b_inner, "b_inner")):
        _dev(t, n)
    b, h, w, c = prev_nhwc.shape
    cl = lat_nhwc.shape[-1]
    if c != 32 or tuple(lat_nhwc.shape) != (b, 2 * h, 2 * w, cl) or not prev_nhwc.is_contiguous() \
            or not lat_nhwc.is_contiguous():
        raise ValueError("fpn_merge: expects contiguous prev [B,h,w,32] and lat [B,2h,2w,cl]")
    out = torch.empty(b, 2 * h, 2 * w, 32, device=prev_nhwc.device)
    with _Span("tmvs_fpn_merge"):
        _lib.check(_lib_h().tmvs_fpn_merge(_ptr(prev_nhwc), _ptr(lat_nhwc), cl, _ptr(w_inner), _ptr(b_inner), b, h, w,
                                           _ptr(out), _stream()), "tmvs_fpn_merge")
    return out


def conv2d_pack(weight):
    """HOST packing of a Conv2d weight [Co][Ci][k][k] into tmvs_conv2d_bn_relu's k-block order."""
    w = np.ascontiguousarray(weight.detach().float().cpu().numpy(), np.float32)
    co, ci, k, _ = w.shape
    out = np.empty(_lib_h().tmvs_conv2d_packed_floats(co, ci, k), np.float32)
    _lib.check(_lib_h().tmvs_conv2d_pack(w.ctypes.data, co, ci, k, out.ctypes.data), "tmvs_conv2d_pack")
    return torch.from_numpy(out)


def conv2d_bn_relu(x, w_packed, cout, k, stride, bn=None, relu=True, nchw_input=False):
    """Conv2d(k, stride, padding k//2, no bias) + folded BN + ReLU (models/module.py:24-61) -> NHWC.
    x: NHWC [B,H,W,Ci], or the NCHW image [B,3,H,W] with nchw_input=True."""
    _dev(x, "x")
    _dev(w_packed, "w_packed")
    if not x.is_contiguous():
        raise ValueError("conv2d_bn_relu: expects a contiguous input")
    if nchw_input:
        b, cin, h, w = x.shape
    else:
        b, h, w, cin = x.shape
    pad = k // 2
    ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    out = torch.empty(b, ho, wo, cout, device=x.device)
    alpha, shift = bn if bn is not None else (None, None)
    with _Span("tmvs_conv2d_bn_relu"):
        _lib.check(_lib_h().tmvs_conv2d_bn_relu(_ptr(x), b, cin, h, w, _ptr(w_packed), cout, k, stride, _ptr(alpha),
                                                _ptr(shift), int(relu), _ptr(out), _stream()), "tmvs_conv2d_bn_relu")
    return out


def entropy_loss(prob, depth_values, depth_gt, mask, grad_scale=0.0, want_grad=False):
    """One stage's entropy_loss (models/module.py:495-531) + smooth-L1 depth loss (:549), and with
    want_grad the gradient of grad_scale * loss w.r.t. the stage's softmax logits.
    Returns (loss [], depth_loss [], wta_depth [B,H,W], photo_conf [B,H,W], grad_logits or None)."""
    for t, n in ((prob, "prob"), (depth_values, "depth_values"), (depth_gt, "depth_gt"), (mask, "mask")):
        _dev(t, n)
    b, d, h, w = prob.shape
    if depth_values.dim() == 4:
        if tuple(depth_values.shape) != (b, d, h, w):
            raise ValueError("depth_values must be [B,D,H,W] or [B,D]")
        per_pixel = 1
    elif tuple(depth_values.shape) == (b, d):
        per_pixel = 0
    else:
        raise ValueError("depth_values must be [B,D,H,W] or [B,D]")
    if tuple(depth_gt.shape) != (b, h, w) or tuple(mask.shape) != (b, h, w):
        raise ValueError("depth_gt and mask must be [B,H,W]")
    nbytes = _lib_h().tmvs_entropy_loss_workspace(b, h, w)
    ws = torch.empty(nbytes // 4 + 64, device=prob.device)
    out = torch.empty(2, device=prob.device)
    wta = torch.empty(b, h, w, device=prob.device)
    conf = torch.empty_like(wta)
    grad = torch.empty_like(prob) if want_grad else None
    with _Span("tmvs_entropy_loss"):
        _lib.check(_lib_h().tmvs_entropy_loss(_ptr(prob), _ptr(depth_values), per_pixel, _ptr(depth_gt), _ptr(mask), b,
                                              d, h, w, ctypes.c_float(grad_scale), _ptr(ws), ws.numel() * 4,
                                              _ptr(out), _ptr(wta), _ptr(conf), _ptr(grad), _stream()),
                   "tmvs_entropy_loss")
    return out[0], out[1], wta, conf, grad


def depth_metrics(depth, depth_gt, mask, depth_interval):
    """focal_loss_bld's epe / less1 / less3 (models/module.py:581-587) -> tensor [3]."""
    for t, n in ((depth, "depth"), (depth_gt, "depth_gt"), (mask, "mask")):
        _dev(t, n)
    if depth.shape != depth_gt.shape or depth.shape != mask.shape:
        raise ValueError("depth, depth_gt and mask must have one shape")
    n = depth.numel()
    nbytes = _lib_h().tmvs_depth_metrics_workspace(n)
    ws = torch.empty(nbytes // 4 + 64, device=depth.device)
    out = torch.empty(3, device=depth.device)
    with _Span("tmvs_depth_metrics"):
        _lib.check(_lib_h().tmvs_depth_metrics(_ptr(depth), _ptr(depth_gt), _ptr(mask), n,
                                               ctypes.c_float(float(depth_interval)), _ptr(ws), ws.numel() * 4,
                                               _ptr(out), _stream()), "tmvs_depth_metrics")
    return out


for _name in ("stage_hypotheses", "warp_corr", "aggregate_finalize", "homo_warping", "softmax_wta", "costregnet",
              "costregnet_wta",
              "conv3d_bn_relu", "deconv3d_bn_relu_add", "fmt_embed", "fmt_kv", "fmt_apply", "fmt_pathway",
              "fmt_forward", "depth_stage", "deform_conv2d", "dcn_fused", "conv3x3_nhwc", "fpn_merge",
              "conv2d_bn_relu", "entropy_loss", "depth_metrics"):
    globals()[_name] = _on_tensor_device(globals()[_name])
del _name


# ----------------------------------------------------------------- CostRegNet training (train.py)
def conv3d_generic(x, w_packed, cout, out_dhw, stride, transposed=False, out=None):
    """tmvs_conv3d_generic: x NDHWC [B,D,H,W,Cin], w_packed [27][cout][Cin] -> y [B,*out_dhw,cout]
    (accumulated into `out` when given)."""
    _dev(x, "x")
    _dev(w_packed, "w_packed")
    b, d, h, w, cin = x.shape
    flags = (_lib.CONV_TRANSPOSED if transposed else 0) | (_lib.CONV_ACCUMULATE if out is not None else 0)
    y = torch.empty(b, *out_dhw, cout, device=x.device) if out is None else out
    if tuple(y.shape) != (b, *out_dhw, cout) or not y.is_contiguous():
        raise ValueError("conv3d_generic: out must be a contiguous [B, D, H, W, cout] tensor")
    with _Span("tmvs_conv3d_generic"):
        _lib.check(_lib_h().tmvs_conv3d_generic(_ptr(x), b, cin, d, h, w, _ptr(w_packed), cout, out_dhw[0], out_dhw[1],
                                                out_dhw[2], stride, flags, _ptr(y), _stream()), "tmvs_conv3d_generic")
    return y


# (cin, cout, stride) of the inference layers' MFMA kernels (tmvs_conv3d_mfma); transposed: (cin, cout)
MFMA_CONV = {(16, 16, 1), (32, 32, 1), (64, 64, 1), (8, 16, 2), (16, 32, 2), (32, 64, 2), (1, 8, 1), (8, 1, 1)}
MFMA_DECONV = {(64, 32), (32, 16), (16, 8)}


def prob_pack(w27):
    """[27][1][8] (tap = kd*9 + kh*3 + kw) -> prob_kernel's [3][72] packing (model.CostRegNet.packed):
    per kh, the {kd=1, kd=2} pairs in (kw, c) order, then kd=0 in (kw, c) order."""
    pw = w27.reshape(3, 3, 3, 8).permute(3, 0, 1, 2)  # [c][kd][kh][kw]
    pairs = pw[:, 1:3].permute(2, 3, 0, 1).reshape(3, -1)
    single = pw[:, 0].permute(1, 2, 0).reshape(3, -1)
    return torch.cat([pairs, single], 1).contiguous()


def conv3d_mfma(x, w_packed, cout, stride, transposed=False, skip=None):
    """tmvs_conv3d_mfma: x NDHWC [B,D,H,W,Cin], w_packed [27][cout][Cin] -> y [B,D',H',W',cout], the raw
    convolution (no BN / ReLU) on the inference MFMA kernels; transposed = ConvTranspose3d k3 s2 p1 op1
    (+ skip, a separate [B,2D,2H,2W,cout] tensor)."""
    _dev(x, "x")
    _dev(w_packed, "w_packed")
    _dev(skip, "skip")
    b, d, h, w, cin = x.shape
    if transposed:
        dims = (2 * d, 2 * h, 2 * w)
    else:
        dims = (d, h, w) if stride == 1 else ((d - 1) // 2 + 1, (h - 1) // 2 + 1, (w - 1) // 2 + 1)
    y = torch.empty(b, *dims, cout, device=x.device)
    if skip is not None and (tuple(skip.shape) != tuple(y.shape) or not skip.is_contiguous()):
        raise ValueError("conv3d_mfma: skip must be a contiguous tensor of the output's shape")
    if (cin, cout) == (8, 1):
        if tuple(w_packed.shape) != (3, 72):
            raise ValueError("conv3d_mfma: the 8 -> 1 conv takes the prob packing [3, 72] (prob_pack)")
    elif tuple(w_packed.shape) != (27, cout, cin):
        raise ValueError("conv3d_mfma: w_packed must be [27, cout, cin]")
    with _Span("tmvs_conv3d_mfma"):
        _lib.check(_lib_h().tmvs_conv3d_mfma(_ptr(x.contiguous()), b, cin, d, h, w, _ptr(w_packed), cout, stride,
                                             int(transposed), _ptr(skip), _ptr(y), _stream()), "tmvs_conv3d_mfma")
    return y


def conv3d_wgrad(direct, gathered, stride):
    """tmvs_conv3d_wgrad: direct [B,pd,ph,pw,A], gathered [B,gd,gh,gw,BC] -> dw [27][A][BC]."""
    _dev(direct, "direct")
    _dev(gathered, "gathered")
    b, pd, ph, pw, a = direct.shape
    _, gd, gh, gw, bc = gathered.shape
    nbytes = _lib_h().tmvs_conv3d_wgrad_workspace(b, pd, ph, pw, a, bc)
    ws = torch.empty(nbytes // 4 + 64, device=direct.device)
    dw = torch.empty(27, a, bc, device=direct.device)
    with _Span("tmvs_conv3d_wgrad"):
        _lib.check(_lib_h().tmvs_conv3d_wgrad(_ptr(direct), a, b, pd, ph, pw, _ptr(gathered), bc, gd, gh, gw, stride,
                                              _ptr(ws), ws.numel() * 4, _ptr(dw), _stream()), "tmvs_conv3d_wgrad")
    return dw


def _bn_ws(nvox, c, device):
    return torch.empty(_lib_h().tmvs_bn_train_workspace(nvox, c) // 4 + 64, device=device)


def bn_stats(z):
    """tmvs_bn_stats: z [..., C] -> (batch mean [C], biased variance [C])."""
    _dev(z, "z")
    c = z.shape[-1]
    nvox = z.numel() // c
    ws = _bn_ws(nvox, c, z.device)
    mean = torch.empty(c, device=z.device)
    var = torch.empty(c, device=z.device)
    with _Span("tmvs_bn_stats"):
        _lib.check(_lib_h().tmvs_bn_stats(_ptr(z), nvox, c, _ptr(ws), ws.numel() * 4, _ptr(mean), _ptr(var), _stream()),
                   "tmvs_bn_stats")
    return mean, var


def bn_relu_train(z, mean, var, gamma, beta, eps, skip=None, out=None):
    """tmvs_bn_relu_train: relu(BN_batch(z)) [+ skip], z [..., C] (written into `out` when given)."""
    for t, n in ((z, "z"), (mean, "mean"), (var, "var"), (gamma, "gamma"), (beta, "beta"), (skip, "skip"), (out, "out")):
        _dev(t, n)
    c = z.shape[-1]
    out = torch.empty_like(z) if out is None else out
    with _Span("tmvs_bn_relu_train"):
        _lib.check(_lib_h().tmvs_bn_relu_train(_ptr(z), z.numel() // c, c, _ptr(mean), _ptr(var), _ptr(gamma),
                                               _ptr(beta), ctypes.c_float(eps), _ptr(skip), _ptr(out), _stream()),
                   "tmvs_bn_relu_train")
    return out


def bn_relu_backward(dy, z, mean, var, gamma, beta, eps, dz=None):
    """tmvs_bn_relu_backward -> (dz, dgamma, dbeta) (dz written into `dz` when given)."""
    for t, n in ((dy, "dy"), (z, "z"), (mean, "mean"), (var, "var"), (gamma, "gamma"), (beta, "beta"), (dz, "dz")):
        _dev(t, n)
    c = z.shape[-1]
    nvox = z.numel() // c
    ws = _bn_ws(nvox, c, z.device)
    dz = torch.empty_like(z) if dz is None else dz
    dg = torch.empty(c, device=z.device)
    db = torch.empty(c, device=z.device)
    with _Span("tmvs_bn_relu_backward"):
        _lib.check(_lib_h().tmvs_bn_relu_backward(_ptr(dy), _ptr(z), nvox, c, _ptr(mean), _ptr(var), _ptr(gamma),
                                                  _ptr(beta), ctypes.c_float(eps), _ptr(ws), ws.numel() * 4, _ptr(dz),
                                                  _ptr(dg), _ptr(db), _stream()), "tmvs_bn_relu_backward")
    return dz, dg, db


def bn_stats_grouped(z):
    """tmvs_bn_stats_grouped: z [G, ..., C] -> (mean [G, C], biased variance [G, C]), statistics per group."""
    _dev(z, "z")
    g, c = z.shape[0], z.shape[-1]
    nvox = z.numel() // (g * c)
    ws = torch.empty(_lib_h().tmvs_bn_train_workspace_grouped(g, nvox, c) // 4 + 64, device=z.device)
    mean = torch.empty(g, c, device=z.device)
    var = torch.empty(g, c, device=z.device)
    with _Span("tmvs_bn_stats_grouped"):
        _lib.check(_lib_h().tmvs_bn_stats_grouped(_ptr(z), g, nvox, c, _ptr(ws), ws.numel() * 4, _ptr(mean), _ptr(var),
                                                  _stream()), "tmvs_bn_stats_grouped")
    return mean, var


def bn_relu_train_grouped(z, mean, var, gamma, beta, eps):
    """tmvs_bn_relu_train_grouped: relu(BN_batch(z)) per group, z [G, ..., C], mean / var [G, C]."""
    for t, n in ((z, "z"), (mean, "mean"), (var, "var"), (gamma, "gamma"), (beta, "beta")):
        _dev(t, n)
    g, c = z.shape[0], z.shape[-1]
    out = torch.empty_like(z)
    with _Span("tmvs_bn_relu_train_grouped"):
        _lib.check(_lib_h().tmvs_bn_relu_train_grouped(_ptr(z), g, z.numel() // (g * c), c, _ptr(mean), _ptr(var),
                                                       _ptr(gamma), _ptr(beta), ctypes.c_float(eps), None, _ptr(out),
                                                       _stream()), "tmvs_bn_relu_train_grouped")
    return out


def bn_relu_backward_grouped(dy, z, mean, var, gamma, beta, eps):
    """tmvs_bn_relu_backward_grouped -> (dz, dgamma, dbeta), dgamma / dbeta summed over the groups in order."""
    for t, n in ((dy, "dy"), (z, "z"), (mean, "mean"), (var, "var"), (gamma, "gamma"), (beta, "beta")):
        _dev(t, n)
    g, c = z.shape[0], z.shape[-1]
    nvox = z.numel() // (g * c)
    ws = torch.empty(_lib_h().tmvs_bn_train_workspace_grouped(g, nvox, c) // 4 + 64, device=z.device)
    dz = torch.empty_like(z)
    dg = torch.empty(c, device=z.device)
    db = torch.empty(c, device=z.device)
    with _Span("tmvs_bn_relu_backward_grouped"):
        _lib.check(_lib_h().tmvs_bn_relu_backward_grouped(_ptr(dy), _ptr(z), g, nvox, c, _ptr(mean), _ptr(var),
                                                          _ptr(gamma), _ptr(beta), ctypes.c_float(eps), _ptr(ws),
                                                          ws.numel() * 4, _ptr(dz), _ptr(dg), _ptr(db), _stream()),
                   "tmvs_bn_relu_backward_grouped")
    return dz, dg, db


def warp_corr_backward(ref_nhwc, src_nhwc, proj12, hyp, dsim, rot_order="auto", planes=False):
    """tmvs_warp_corr_backward: one sample, ref [H,W,C], src [V,H,W,C] NHWC, proj12 HOST [V,12],
    hyp [D,H,W], dsim [V,D,H,W] -> (dref [H,W,C], dsrc [V,H,W,C], flag tensor [1] int32: bit 0 a
    non-finite dsim / ref, bit 1 non-planar hyp under planes=True). planes=True (TMVS_WARP_BWD_PLANES:
    hyp[d] is one depth per plane, stage 1) gathers dsrc per source texel instead of scattering it."""
    for t, n in ((ref_nhwc, "ref"), (src_nhwc, "src"), (hyp, "hyp"), (dsim, "dsim")):
        _dev(t, n)
    v, h, w, c = src_nhwc.shape
    d = hyp.shape[0]
    if tuple(dsim.shape) != (v, d, h, w) or tuple(ref_nhwc.shape) != (h, w, c):
        raise ValueError("warp_corr_backward: shapes must be ref [H,W,C], src [V,H,W,C], hyp [D,H,W], dsim [V,D,H,W]")
    proj = np.ascontiguousarray(proj12, np.float32).reshape(v, 12)
    nbytes = _lib_h().tmvs_warp_corr_backward_workspace(v, c, h, w, hyp.shape[0])
    ws = torch.empty(nbytes // 4 + 64, device=hyp.device)
    dref = torch.empty_like(ref_nhwc)
    dsrc = torch.empty_like(src_nhwc)
    with _Span("tmvs_warp_corr_backward"):
        _lib.check(_lib_h().tmvs_warp_corr_backward(_ptr(ref_nhwc), _ptr(src_nhwc), proj.ctypes.data, _ptr(hyp), _ptr(dsim),
                                                    v, c, d, h, w,
                                                    warp_flags(rot_order, h * w) | (_lib.WARP_BWD_PLANES if planes else 0), _ptr(ws),
                                                    ws.numel() * 4, _ptr(dref), _ptr(dsrc), _stream()),
                   "tmvs_warp_corr_backward")
    flag = ws.view(torch.int32)[2 * v * h * w * c: 2 * v * h * w * c + 1]
    return dref, dsrc, flag


def pixelwise_train_forward(sims, pwp):
    """tmvs_pixelwise_train_forward: sims [V,D,H,W], pwp [201] -> (stats [V,48], view_w [V,H,W], dstar int32)."""
    _dev(sims, "sims")
    _dev(pwp, "pwp")
    v, d, h, w = sims.shape
    ws = torch.empty(_lib_h().tmvs_pixelwise_train_workspace() // 4 + 64, device=sims.device)
    stats = torch.empty(v, 48, device=sims.device)
    vw = torch.empty(v, h, w, device=sims.device)
    dstar = torch.empty(v, h, w, device=sims.device, dtype=torch.int32)
    with _Span("tmvs_pixelwise_train_forward"):
        _lib.check(_lib_h().tmvs_pixelwise_train_forward(_ptr(sims), v, d, h, w, _ptr(pwp), _ptr(ws), ws.numel() * 4,
                                                         _ptr(stats), _ptr(vw), _ptr(dstar), _stream()),
                   "tmvs_pixelwise_train_forward")
    return stats, vw, dstar


def aggregate_train(sims, view_w, vw_shift):
    """tmvs_aggregate_train: sims [V,D,H,W], view_w [V,H>>s,W>>s] -> (sim [D,H,W], wsum [H,W])."""
    _dev(sims, "sims")
    _dev(view_w, "view_w")
    v, d, h, w = sims.shape
    sim = torch.empty(d, h, w, device=sims.device)
    wsum = torch.empty(h, w, device=sims.device)
    with _Span("tmvs_aggregate_train"):
        _lib.check(_lib_h().tmvs_aggregate_train(_ptr(sims), _ptr(view_w), v, d, h, w, vw_shift, _ptr(sim), _ptr(wsum),
                                                 _stream()), "tmvs_aggregate_train")
    return sim, wsum


def aggregate_train_backward(dsim, sims, sim, wsum, view_w, vw_shift, want_dview_w):
    """tmvs_aggregate_train_backward -> (dsims [V,D,H,W], dview_w [V,H,W] or None)."""
    for t, n in ((dsim, "dsim"), (sims, "sims"), (sim, "sim"), (wsum, "wsum"), (view_w, "view_w")):
        _dev(t, n)
    v, d, h, w = sims.shape
    dsims = torch.empty_like(sims)
    dvw = torch.empty(v, h, w, device=sims.device) if want_dview_w else None
    with _Span("tmvs_aggregate_train_backward"):
        _lib.check(_lib_h().tmvs_aggregate_train_backward(_ptr(dsim), _ptr(sims), _ptr(sim), _ptr(wsum), _ptr(view_w), v,
                                                          d, h, w, vw_shift, _ptr(dsims), _ptr(dvw), _stream()),
                   "tmvs_aggregate_train_backward")
    return dsims, dvw


def pixelwise_train_backward(sims, pwp, stats, view_w, dstar, dview_w, dsims):
    """tmvs_pixelwise_train_backward: adds the PixelwiseNet path into dsims (in place) -> dpwp [201]."""
    for t, n in ((sims, "sims"), (pwp, "pwp"), (stats, "stats"), (view_w, "view_w"), (dview_w, "dview_w"),
                 (dsims, "dsims")):
        _dev(t, n)
    v, d, h, w = sims.shape
    ws = torch.empty(_lib_h().tmvs_pixelwise_train_workspace() // 4 + 64, device=sims.device)
    dpwp = torch.zeros(201, device=sims.device)
    with _Span("tmvs_pixelwise_train_backward"):
        _lib.check(_lib_h().tmvs_pixelwise_train_backward(_ptr(sims), v, d, h, w, _ptr(pwp), _ptr(stats), _ptr(view_w),
                                                          _ptr(dstar), _ptr(dview_w), _ptr(ws), ws.numel() * 4,
                                                          _ptr(dsims), _ptr(dpwp), _stream()),
                   "tmvs_pixelwise_train_backward")
    return dpwp


def upsample2_add_nhwc(r, lateral_nchw):
    """tmvs_upsample2_add_nhwc: r [N,h,w,C] -> bilinear x2 + lateral [N,C,2h,2w] -> [N,2h,2w,C]."""
    _dev(r, "r")
    _dev(lateral_nchw, "lateral")
    n, h, w, c = r.shape
    if tuple(lateral_nchw.shape) != (n, c, 2 * h, 2 * w):
        raise ValueError("upsample2_add_nhwc: lateral must be [N, C, 2h, 2w]")
    u = torch.empty(n, 2 * h, 2 * w, c, device=r.device)
    with _Span("tmvs_upsample2_add_nhwc"):
        _lib.check(_lib_h().tmvs_upsample2_add_nhwc(_ptr(r), _ptr(lateral_nchw), n, h, w, c, _ptr(u), _stream()),
                   "tmvs_upsample2_add_nhwc")
    return u


def upsample2_backward_nhwc(du):
    """tmvs_upsample2_backward_nhwc: du [N,2h,2w,C] -> dr [N,h,w,C]."""
    _dev(du, "du")
    n, hh, ww, c = du.shape
    dr = torch.empty(n, hh // 2, ww // 2, c, device=du.device)
    with _Span("tmvs_upsample2_backward_nhwc"):
        _lib.check(_lib_h().tmvs_upsample2_backward_nhwc(_ptr(du), n, hh // 2, ww // 2, c, _ptr(dr), _stream()),
                   "tmvs_upsample2_backward_nhwc")
    return dr


def _tokens(x, name, c=None):
    _dev(x, name)
    if x.dim() != 2 or (c is not None and x.shape[1] != c):
        raise ValueError(f"{name}: expected a [T, {c or 'C'}] token matrix, got {tuple(x.shape)}")
    return x.shape[0]


def token_linear(x, w, b=None, transpose_w=False, relu_of=None, out=None, residual=None):
    """tmvs_token_linear: x [T,in] -> x w^T + b (w [out,in]) or, transpose_w, x w (w [in',out'] -> out = in').

    relu_of [T,out] masks the result where relu_of <= 0; out (given) is accumulated into; residual (given,
    tmvs_token_linear_res) -> a new residual + result (the same additions as out=residual.clone())."""
    t = _tokens(x, "x")
    for a, n in ((w, "w"), (b, "b"), (relu_of, "relu_of"), (out, "out"), (residual, "residual")):
        _dev(a, n)
    if residual is not None:
        if out is not None:
            raise ValueError("token_linear: give out or residual, not both")
        o_f = w.shape[0] if not transpose_w else w.shape[1]
        if x.shape[1] != (w.shape[1] if not transpose_w else w.shape[0]) or tuple(residual.shape) != (t, o_f) or \
                (relu_of is not None and tuple(relu_of.shape) != (t, o_f)):
            raise ValueError("token_linear: shape mismatch")
        y = torch.empty(t, o_f, device=x.device)
        with _Span("tmvs_token_linear_res"):
            _lib.check(_lib_h().tmvs_token_linear_res(_ptr(x), t, x.shape[1], o_f, _ptr(w),
                                                      _ptr(b) if b is not None else None, int(transpose_w),
                                                      _ptr(relu_of) if relu_of is not None else None, _ptr(residual),
                                                      _ptr(y), _stream()), "tmvs_token_linear_res")
        return y
    o_f = w.shape[0] if not transpose_w else w.shape[1]
    if x.shape[1] != (w.shape[1] if not transpose_w else w.shape[0]):
        raise ValueError("token_linear: x / w feature mismatch")
    acc = out is not None
    for a, n in ((relu_of, "relu_of"), (out, "out")):
        if a is not None and tuple(a.shape) != (t, o_f):
            raise ValueError(f"token_linear: {n} must be [{t}, {o_f}]")
    y = out if acc else torch.empty(t, o_f, device=x.device)
    with _Span("tmvs_token_linear"):
        _lib.check(_lib_h().tmvs_token_linear(_ptr(x), t, x.shape[1], o_f, _ptr(w), _ptr(b) if b is not None else None,
                                              int(transpose_w), _ptr(relu_of) if relu_of is not None else None, int(acc),
                                              _ptr(y), _stream()), "tmvs_token_linear")
    return y


def token_wgrad(dy, x, dw=None, db=None):
    """tmvs_token_wgrad: dy [T,a], x [T,b] -> (dw [a,b] = dy^T x, db [a] = column sums of dy); accumulates into
    dw/db when both are given."""
    t = _tokens(dy, "dy")
    if _tokens(x, "x") != t:
        raise ValueError("token_wgrad: token counts differ")
    a, b = dy.shape[1], x.shape[1]
    acc = dw is not None
    if acc != (db is not None):
        raise ValueError("token_wgrad: give both dw and db or neither")
    if not acc:
        dw, db = torch.empty(a, b, device=dy.device), torch.empty(a, device=dy.device)
    for z, n, shp in ((dw, "dw", (a, b)), (db, "db", (a,))):
        _dev(z, n)
        if tuple(z.shape) != shp:
            raise ValueError(f"token_wgrad: {n} must be {shp}")
    ws = torch.empty(_lib_h().tmvs_token_wgrad_workspace(t, a, b) // 4 + 64, device=dy.device)
    with _Span("tmvs_token_wgrad"):
        _lib.check(_lib_h().tmvs_token_wgrad(_ptr(dy), a, _ptr(x), b, t, _ptr(ws), ws.numel() * 4, _ptr(dw), _ptr(db),
                                             int(acc), _stream()), "tmvs_token_wgrad")
    return dw, db


def layer_norm_fwd(x, g, b):
    """tmvs_layer_norm_fwd: LayerNorm(32) of x [T,32]."""
    t = _tokens(x, "x", 32)
    _dev(g, "g")
    _dev(b, "b")
    y = torch.empty_like(x)
    with _Span("tmvs_layer_norm_fwd"):
        _lib.check(_lib_h().tmvs_layer_norm_fwd(_ptr(x), t, _ptr(g), _ptr(b), _ptr(y), _stream()), "tmvs_layer_norm_fwd")
    return y


def layer_norm_bwd(dy, x, g, dgb=None):
    """tmvs_layer_norm_bwd: -> (dx [T,32], dgb [64] = dgamma | dbeta); accumulates into dgb when given."""
    t = _tokens(dy, "dy", 32)
    if _tokens(x, "x", 32) != t:
        raise ValueError("layer_norm_bwd: token counts differ")
    _dev(g, "g")
    _dev(dgb, "dgb")
    acc = dgb is not None
    dgb = dgb if acc else torch.empty(64, device=dy.device)
    dx = torch.empty_like(dy)
    ws = torch.empty(_lib_h().tmvs_layer_norm_bwd_workspace(t) // 4 + 64, device=dy.device)
    with _Span("tmvs_layer_norm_bwd"):
        _lib.check(_lib_h().tmvs_layer_norm_bwd(_ptr(dy), _ptr(x), t, _ptr(g), _ptr(ws), ws.numel() * 4, _ptr(dx),
                                                _ptr(dgb), int(acc), _stream()), "tmvs_layer_norm_bwd")
    return dx, dgb


def linattn_fwd(q, kv, tokens_per_group):
    """tmvs_linattn_fwd: q [T,32] (pre-elu), kv [G,160] (G == 1: shared) -> msg [T,32]."""
    t = _tokens(q, "q", 32)
    _dev(kv, "kv")
    msg = torch.empty_like(q)
    stride = 0 if kv.shape[0] == 1 else _lib.KV_NFLOATS
    with _Span("tmvs_linattn_fwd"):
        _lib.check(_lib_h().tmvs_linattn_fwd(_ptr(q), t, tokens_per_group, _ptr(kv), stride, _ptr(msg), _stream()),
                   "tmvs_linattn_fwd")
    return msg


def linattn_bwd_q(q, dmsg, kv, tokens_per_group):
    """tmvs_linattn_bwd_q: -> (dq [T,32], dkv [T / tokens_per_group, 160])."""
    t = _tokens(q, "q", 32)
    if _tokens(dmsg, "dmsg", 32) != t:
        raise ValueError("linattn_bwd_q: token counts differ")
    if t % tokens_per_group:
        raise ValueError("linattn_bwd_q: tokens must be a multiple of tokens_per_group")
    _dev(kv, "kv")
    groups = t // tokens_per_group
    stride = 0 if kv.shape[0] == 1 else _lib.KV_NFLOATS
    if stride and kv.shape[0] != groups:
        raise ValueError("linattn_bwd_q: kv must have one row per group (or one shared row)")
    dq = torch.empty_like(q)
    dkv = torch.empty(groups, _lib.KV_NFLOATS, device=q.device)
    ws = torch.empty(_lib_h().tmvs_linattn_bwd_workspace(t, tokens_per_group) // 4 + 64, device=q.device)
    with _Span("tmvs_linattn_bwd_q"):
        _lib.check(_lib_h().tmvs_linattn_bwd_q(_ptr(q), _ptr(dmsg), t, tokens_per_group, _ptr(kv), stride, _ptr(ws),
                                               ws.numel() * 4, _ptr(dq), _ptr(dkv), _stream()), "tmvs_linattn_bwd_q")
    return dq, dkv


def linattn_bwd_kv(k, v, dkv, tokens_per_group):
    """tmvs_linattn_bwd_kv: k (pre-elu), v [S,32], dkv [S / tokens_per_group, 160] -> (dk, dv)."""
    s = _tokens(k, "k", 32)
    if _tokens(v, "v", 32) != s or dkv.shape[0] * tokens_per_group != s:
        raise ValueError("linattn_bwd_kv: shape mismatch")
    _dev(dkv, "dkv")
    dk, dv = torch.empty_like(k), torch.empty_like(v)
    with _Span("tmvs_linattn_bwd_kv"):
        _lib.check(_lib_h().tmvs_linattn_bwd_kv(_ptr(k), _ptr(v), s, tokens_per_group, _ptr(dkv), _ptr(dk), _ptr(dv),
                                                _stream()), "tmvs_linattn_bwd_kv")
    return dk, dv


def adam_step(param_flat, grad_flat, exp_avg, exp_avg_sq, lr, betas, eps, weight_decay, step):
    """tmvs_adam_step: one Adam update (torch's order) of a flat fp32 parameter buffer, in place."""
    for t, n in ((param_flat, "param"), (grad_flat, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _dev(t, n)
        if t.numel() != param_flat.numel():
            raise ValueError(f"adam_step: {n} must have {param_flat.numel()} elements")
    with _Span("tmvs_adam_step"):
        _lib.check(_lib_h().tmvs_adam_step(_ptr(param_flat), _ptr(grad_flat), _ptr(exp_avg), _ptr(exp_avg_sq),
                                           param_flat.numel(), float(lr), float(betas[0]), float(betas[1]), float(eps),
                                           float(weight_decay), int(step), _stream()), "tmvs_adam_step")


def adam_step_dev(param_flat, grad_flat, exp_avg, exp_avg_sq, lr, betas, eps, weight_decay, step_counter, scalars,
                  lr_dev=None):
    """tmvs_adam_step_dev: adam_step with the step number advanced on the device (graph-replayable).
    lr_dev: an optional device float64 [1] read by the launch when it runs (a replayed graph then
    follows the value the caller writes there); None = lr by value."""
    for t, n in ((param_flat, "param"), (grad_flat, "grad"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq"),
                 (scalars, "scalars")):
        _dev(t, n)
    if step_counter.dtype != torch.int32 or not step_counter.is_cuda:
        raise RuntimeError("step_counter must be a device int32 tensor")
    if lr_dev is not None and (lr_dev.dtype != torch.float64 or not lr_dev.is_cuda or lr_dev.numel() != 1):
        raise RuntimeError("lr_dev must be a device float64 tensor of one element")
    with _Span("tmvs_adam_step"):
        _lib.check(_lib_h().tmvs_adam_step_dev(_ptr(param_flat), _ptr(grad_flat), _ptr(exp_avg), _ptr(exp_avg_sq),
                                               param_flat.numel(), float(lr),
                                               _ptr(lr_dev), float(betas[0]),
                                               float(betas[1]), float(eps), float(weight_decay), _ptr(step_counter),
                                               _ptr(scalars),
                                               _stream()), "tmvs_adam_step_dev")


for _name in ("conv3d_generic", "conv3d_mfma", "conv3d_wgrad", "bn_stats", "bn_relu_train", "bn_relu_backward", "bn_stats_grouped", "bn_relu_train_grouped",
              "bn_relu_backward_grouped", "warp_corr_backward",
              "upsample2_add_nhwc", "upsample2_backward_nhwc", "pixelwise_train_forward", "aggregate_train", "aggregate_train_backward", "pixelwise_train_backward",
              "token_linear", "token_wgrad", "layer_norm_fwd", "layer_norm_bwd", "linattn_fwd", "linattn_bwd_q",
              "linattn_bwd_kv", "adam_step", "adam_step_dev"):
    globals()[_name] = _on_tensor_device(globals()[_name])
del _name


# ----------------------------------------------------------------- FeatureNet training (featurenet_train.py)
def conv2d_generic(x, w_taps, cout, out_hw, k, stride, pad, bias=None, transposed=False, out=None):
    """tmvs_conv2d_generic: x NHWC [B,H,W,Cin], w_taps [k*k][cout][Cin] -> y [B,*out_hw,cout] (+ bias);
    accumulated into `out` when given."""
    _dev(x, "x")
    _dev(w_taps, "w_taps")
    _dev(bias, "bias")
    b, h, w, cin = x.shape
    flags = (_lib.CONV_TRANSPOSED if transposed else 0) | (_lib.CONV_ACCUMULATE if out is not None else 0)
    y = torch.empty(b, *out_hw, cout, device=x.device) if out is None else out
    if tuple(y.shape) != (b, *out_hw, cout) or not y.is_contiguous():
        raise ValueError("conv2d_generic: out must be a contiguous [B, H, W, cout] tensor")
    with _Span("tmvs_conv2d_generic"):
        _lib.check(_lib_h().tmvs_conv2d_generic(_ptr(x), b, cin, h, w, _ptr(w_taps), _ptr(bias), cout, out_hw[0],
                                                out_hw[1], k, stride, pad, flags, _ptr(y), _stream()),
                   "tmvs_conv2d_generic")
    return y


def conv2d_wgrad(direct, gathered, k, stride, pad):
    """tmvs_conv2d_wgrad: direct [B,ph,pw,A] (dz), gathered [B,gh,gw,BC] (x) -> dw [k*k][A][BC]."""
    _dev(direct, "direct")
    _dev(gathered, "gathered")
    b, ph, pw, a = direct.shape
    _, gh, gw, bc = gathered.shape
    nbytes = _lib_h().tmvs_conv2d_wgrad_workspace(b, ph, pw, a, bc, k)
    ws = torch.empty(nbytes // 4 + 64, device=direct.device)
    dw = torch.empty(k * k, a, bc, device=direct.device)
    with _Span("tmvs_conv2d_wgrad"):
        _lib.check(_lib_h().tmvs_conv2d_wgrad(_ptr(direct), a, b, ph, pw, _ptr(gathered), bc, gh, gw, k, stride, pad,
                                              _ptr(ws), ws.numel() * 4, _ptr(dw), _stream()), "tmvs_conv2d_wgrad")
    return dw


def colsum(x):
    """tmvs_colsum: x [..., C] -> [C] (sum over every other axis; C <= 32)."""
    _dev(x, "x")
    c = x.shape[-1]
    n = x.numel() // c
    ws = torch.empty(_lib_h().tmvs_colsum_workspace(n, c) // 4 + 64, device=x.device)
    out = torch.empty(c, device=x.device)
    with _Span("tmvs_colsum"):
        _lib.check(_lib_h().tmvs_colsum(_ptr(x), n, c, _ptr(ws), ws.numel() * 4, _ptr(out), _stream()), "tmvs_colsum")
    return out


def dcn_forward_train(x_nhwc, wom_packed, bom, w_packed, bias, cout, want_nchw=False):
    """tmvs_dcn_forward_train: DCN.forward without BN/ReLU -> (out_nhwc [B,H,W,cout], offset_mask
    [B,27,H,W], out_nchw or None)."""
    for t, n in ((x_nhwc, "x_nhwc"), (wom_packed, "wom_packed"), (bom, "bom"), (w_packed, "w_packed"), (bias, "bias")):
        _dev(t, n)
    b, h, w, cin = x_nhwc.shape
    out_nhwc = torch.empty(b, h, w, cout, device=x_nhwc.device)
    out = torch.empty(b, cout, h, w, device=x_nhwc.device) if want_nchw else None
    om = torch.empty(b, 27, h, w, device=x_nhwc.device)
    with _Span("tmvs_dcn_forward_train"):
        _lib.check(_lib_h().tmvs_dcn_forward_train(_ptr(x_nhwc), _ptr(wom_packed), _ptr(bom), _ptr(w_packed), _ptr(bias),
                                                   b, cin, cout, h, w, _ptr(out), _ptr(out_nhwc), _ptr(om), _stream()),
                   "tmvs_dcn_forward_train")
    return out_nhwc, om, out


def dcn_backward(x_nhwc, offset_mask, w_taps, dy_nhwc, dx_nhwc):
    """tmvs_dcn_backward: -> (dom [B,H,W,32] (channels 27..31 zero), dw_taps [9][cout][32]); dx_nhwc is
    accumulated into."""
    for t, n in ((x_nhwc, "x_nhwc"), (offset_mask, "offset_mask"), (w_taps, "w_taps"), (dy_nhwc, "dy_nhwc"),
                 (dx_nhwc, "dx_nhwc")):
        _dev(t, n)
    b, h, w, cin = x_nhwc.shape
    cout = dy_nhwc.shape[-1]
    if tuple(offset_mask.shape) != (b, 27, h, w) or tuple(dy_nhwc.shape) != (b, h, w, cout) or \
            tuple(w_taps.shape) != (9, cout, cin) or tuple(dx_nhwc.shape) != tuple(x_nhwc.shape):
        raise ValueError("dcn_backward: shape mismatch")
    ws = torch.empty(_lib_h().tmvs_dcn_backward_workspace(b, cout, h, w) // 4 + 64, device=x_nhwc.device)
    dom = torch.empty(b, h, w, 32, device=x_nhwc.device)
    dw = torch.empty(9, cout, cin, device=x_nhwc.device)
    with _Span("tmvs_dcn_backward"):
        _lib.check(_lib_h().tmvs_dcn_backward(_ptr(x_nhwc), _ptr(offset_mask), _ptr(w_taps), _ptr(dy_nhwc), b, cin, cout,
                                              h, w, _ptr(ws), ws.numel() * 4, _ptr(dx_nhwc), _ptr(dom), _ptr(dw),
                                              _stream()), "tmvs_dcn_backward")
    return dom, dw


_DCN_FAR = {}


def dcn_backward_set(x_nhwc, offset_mask, w_taps, dy_nhwc):
    """tmvs_dcn_backward_set: -> (dx [B,H,W,32] written, not accumulated; dom; dw_taps). The corners beyond the
    LDS windows go through a zeroed far buffer kept per (device, shape) and cleared again by the call, so no
    activation-sized zero fill runs per call. One buffer per shape: an eager call on another stream waits for
    the previous call's stream (event), and the buffer is created outside any HIP-graph capture (raises if a
    shape is first seen while capturing)."""
    for t, n in ((x_nhwc, "x_nhwc"), (offset_mask, "offset_mask"), (w_taps, "w_taps"), (dy_nhwc, "dy_nhwc")):
        _dev(t, n)
    b, h, w, cin = x_nhwc.shape
    cout = dy_nhwc.shape[-1]
    if tuple(offset_mask.shape) != (b, 27, h, w) or tuple(dy_nhwc.shape) != (b, h, w, cout) or \
            tuple(w_taps.shape) != (9, cout, cin):
        raise ValueError("dcn_backward_set: shape mismatch")
    key = (str(x_nhwc.device), tuple(x_nhwc.shape))
    capturing = torch.cuda.is_current_stream_capturing()
    ent = _DCN_FAR.get(key)
    if ent is None:
        if capturing:  # a zero fill recorded in the graph would run per replay, and an eager call before the
            # first replay would read an unfilled buffer: the buffer must exist before the capture
            raise RuntimeError("dcn_backward_set: first call for this shape inside a HIP-graph capture; run one eager "
                               "step first (the far buffer is allocated and zeroed outside any capture)")
        ent = _DCN_FAR[key] = [torch.zeros_like(x_nhwc), None, None]  # buffer, last stream, its done event
    far = ent[0]
    cur = torch.cuda.current_stream(x_nhwc.device)
    if not capturing and ent[1] is not None and ent[1] != cur:  # a call on another stream: order after its use
        cur.wait_event(ent[2])
    ws = torch.empty(_lib_h().tmvs_dcn_backward_workspace(b, cout, h, w) // 4 + 64, device=x_nhwc.device)
    dx = torch.empty_like(x_nhwc)
    dom = torch.empty(b, h, w, 32, device=x_nhwc.device)
    dw = torch.empty(9, cout, cin, device=x_nhwc.device)
    with _Span("tmvs_dcn_backward_set"):
        _lib.check(_lib_h().tmvs_dcn_backward_set(_ptr(x_nhwc), _ptr(offset_mask), _ptr(w_taps), _ptr(dy_nhwc), b, cin,
                                                  cout, h, w, _ptr(ws), ws.numel() * 4, _ptr(dx), _ptr(dom), _ptr(dw),
                                                  _ptr(far), _stream()), "tmvs_dcn_backward_set")
    if not capturing:
        ev = ent[2] or torch.cuda.Event()
        ev.record(cur)
        ent[1], ent[2] = cur, ev
    return dx, dom, dw


def nearest_up2_backward_nhwc(d, out=None):
    """tmvs_nearest_up2_backward_nhwc: d [n,2h,2w,C] -> [n,h,w,C] (accumulated into `out` when given)."""
    _dev(d, "d")
    n, h2, w2, c = d.shape
    y = torch.empty(n, h2 // 2, w2 // 2, c, device=d.device) if out is None else out
    with _Span("tmvs_nearest_up2_backward_nhwc"):
        _lib.check(_lib_h().tmvs_nearest_up2_backward_nhwc(_ptr(d), n, h2 // 2, w2 // 2, c, int(out is not None), _ptr(y),
                                                           _stream()), "tmvs_nearest_up2_backward_nhwc")
    return y


def softmax_backward(prob, dprob):
    """tmvs_softmax_backward: prob, dprob [B,D,H,W] -> d logits."""
    _dev(prob, "prob")
    _dev(dprob, "dprob")
    b, d, h, w = prob.shape
    out = torch.empty_like(prob)
    with _Span("tmvs_softmax_backward"):
        _lib.check(_lib_h().tmvs_softmax_backward(_ptr(prob), _ptr(dprob), b, d, h, w, _ptr(out), _stream()),
                   "tmvs_softmax_backward")
    return out


for _name in ("conv2d_generic", "conv2d_wgrad", "colsum", "dcn_forward_train", "dcn_backward", "dcn_backward_set",
              "conv3x3_nhwc_acc",
              "nearest_up2_backward_nhwc", "softmax_backward"):
    globals()[_name] = _on_tensor_device(globals()[_name])
del _name
