"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the checker / the timed CPU baseline. The
product path (``transmvsnet_amd``) never imports it.

A from-scratch, functional restatement of the TransMVSNet depth-inference forward
(``/root/reference/models``) in PyTorch-CPU fp32. It takes a plain state_dict (the
reference key layout) and runs the SAME ATen ops in the SAME order as the reference
modules, so on identical inputs it is bit-identical to the reference forward
(pinned by ``tests/golden/*.npz``, produced by ``tests/golden/make_golden.py`` from
the real reference imported in the survey container).

Every function cites the reference file:line it follows.
"""
from __future__ import annotations

import math

import einops
import torch
import torch.nn.functional as F

ALIGN_CORNERS_RANGE = False  # models/TransMVSNet.py:8
BN_EPS = 1e-5                # nn.BatchNorm default, models/module.py:132,173,218
LN_EPS = 1e-5                # nn.LayerNorm default, models/FMT.py:91-92
ATTN_EPS = 1e-6              # models/FMT.py:17
FMT_LAYERS = ["self", "cross"] * 4   # models/FMT.py:189
FMT_NHEAD = 8                        # models/FMT.py:188
NDEPTHS = (48, 32, 8)                # models/TransMVSNet.py:113
DEPTH_RATIOS = (4.0, 1.0, 0.5)       # models/TransMVSNet.py:114
STAGE_SCALES = (4, 2, 1)             # models/TransMVSNet.py:128-132
DEPTH_CLAMP = (425.0, 935.0)         # models/TransMVSNet.py:221


# ----------------------------------------------------------------------------- helpers
def _bn(x, sd, p, training=False):
    """nn.BatchNorm{2,3}d (models/module.py:132,173,218): eval mode, or train mode (batch statistics;
    the running statistics in `sd` are updated in place with momentum 0.1 and num_batches_tracked
    counted, as the module does in train mode)."""
    if training and p + "num_batches_tracked" in sd:
        sd[p + "num_batches_tracked"].add_(1)
    return F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"], sd[p + "weight"], sd[p + "bias"],
                        training, 0.1, BN_EPS)


def _lin(x, sd, p):
    return F.linear(x, sd[p + "weight"], sd[p + "bias"])


# ----------------------------------------------------------------------------- FMT
def position_encoding_sine(d_model: int, max_shape=(600, 600)):
    """PositionEncodingSine buffer, models/position_encoding.py:28-52 (temp_bug_fix=True)."""
    pe = torch.zeros((d_model, *max_shape))
    y_pos = torch.ones(max_shape).cumsum(0).float().unsqueeze(0)
    x_pos = torch.ones(max_shape).cumsum(1).float().unsqueeze(0)
    div = torch.exp(torch.arange(0, d_model // 2, 2).float() * (-math.log(10000.0) / (d_model // 2)))
    div = div[:, None, None]
    pe[0::4, :, :] = torch.sin(x_pos * div)
    pe[1::4, :, :] = torch.cos(x_pos * div)
    pe[2::4, :, :] = torch.sin(y_pos * div)
    pe[3::4, :, :] = torch.cos(y_pos * div)
    return pe.unsqueeze(0)


_PE_CACHE = {}


def _pe(d_model):
    if d_model not in _PE_CACHE:
        _PE_CACHE[d_model] = position_encoding_sine(d_model)
    return _PE_CACHE[d_model]


def linear_attention(q, k, v, eps=ATTN_EPS):
    """LinearAttention.forward, models/FMT.py:22-37 (elu+1 feature map)."""
    qf = F.elu(q) + 1
    kf = F.elu(k) + 1
    kv = torch.einsum("nshd,nshm->nhmd", kf, v)
    z = 1 / (torch.einsum("nlhd,nhd->nlh", qf, kf.sum(dim=1)) + eps)
    return torch.einsum("nlhd,nhmd,nlh->nlhm", qf, kv, z).contiguous()


def encoder_layer(sd, p, x, source, nhead=FMT_NHEAD):
    """EncoderLayer.forward (models/FMT.py:96-111) with AttentionLayer (:56-75); dropout p=0."""
    n, l, _ = x.shape
    s = source.shape[1]
    q = _lin(x, sd, p + "attention.query_projection.").view(n, l, nhead, -1)
    k = _lin(source, sd, p + "attention.key_projection.").view(n, s, nhead, -1)
    v = _lin(source, sd, p + "attention.value_projection.").view(n, s, nhead, -1)
    msg = linear_attention(q, k, v).view(n, l, -1)
    x = x + _lin(msg, sd, p + "attention.out_projection.")
    d = x.shape[-1]
    x = F.layer_norm(x, (d,), sd[p + "norm1.weight"], sd[p + "norm1.bias"], LN_EPS)
    y = F.relu(_lin(x, sd, p + "linear1."))
    y = _lin(y, sd, p + "linear2.")
    return F.layer_norm(x + y, (d,), sd[p + "norm2.weight"], sd[p + "norm2.bias"], LN_EPS)


def fmt_ref(sd, ref_stage1, prefix="FMT_with_pathway.FMT."):
    """FMT.forward(feat='ref'), models/FMT.py:147-159: PE, then the 4 self layers."""
    h = ref_stage1.shape[2]
    x = ref_stage1 + _pe(ref_stage1.shape[1])[:, :, :ref_stage1.size(2), :ref_stage1.size(3)]
    x = einops.rearrange(x, "n c h w -> n (h w) c")
    outs = []
    for i, name in enumerate(FMT_LAYERS):
        if name == "self":
            x = encoder_layer(sd, f"{prefix}layers.{i}.", x, x)
            outs.append(einops.rearrange(x, "n (h w) c -> n c h w", h=h))
    return outs


def fmt_src(sd, ref_list, src_stage1, prefix="FMT_with_pathway.FMT."):
    """FMT.forward(feat='src'), models/FMT.py:161-177: self / cross(ref_list[i//2]) alternation."""
    h = ref_list[0].shape[2]
    refs = [einops.rearrange(r, "n c h w -> n (h w) c") for r in ref_list]
    x = src_stage1 + _pe(src_stage1.shape[1])[:, :, :src_stage1.size(2), :src_stage1.size(3)]
    x = einops.rearrange(x, "n c h w -> n (h w) c")
    for i, name in enumerate(FMT_LAYERS):
        if name == "self":
            x = encoder_layer(sd, f"{prefix}layers.{i}.", x, x)
        else:
            x = encoder_layer(sd, f"{prefix}layers.{i}.", x, refs[i // 2])
    return einops.rearrange(x, "n (h w) c -> n c h w", h=h)


def _upsample_add(x, y):
    """FMT_with_pathway._upsample_add, models/FMT.py:201-209 (bilinear, align_corners=False)."""
    _, _, h, w = y.size()
    return F.interpolate(x, size=(h, w), mode="bilinear") + y


def fmt_with_pathway(sd, features, prefix="FMT_with_pathway."):
    """FMT_with_pathway.forward, models/FMT.py:212-230. Returns NEW per-view dicts."""
    out = []
    ref_list = None
    for v, f in enumerate(features):
        g = dict(f)
        if v == 0:
            ref_list = fmt_ref(sd, f["stage1"].clone(), prefix + "FMT.")
            g["stage1"] = ref_list[-1]
        else:
            g["stage1"] = fmt_src(sd, [r.clone() for r in ref_list], f["stage1"].clone(), prefix + "FMT.")
        g["stage2"] = F.conv2d(_upsample_add(F.conv2d(g["stage1"], sd[prefix + "dim_reduction_1.weight"]), f["stage2"]),
                               sd[prefix + "smooth_1.weight"], padding=1)
        g["stage3"] = F.conv2d(_upsample_add(F.conv2d(g["stage2"], sd[prefix + "dim_reduction_2.weight"]), f["stage3"]),
                               sd[prefix + "smooth_2.weight"], padding=1)
        out.append(g)
    return out


# ----------------------------------------------------------------------------- warp / cost volume
def compose_proj(proj):
    """[B,2,4,4] (extrinsic, intrinsic) -> [B,4,4] K*E in rows 0..2, models/TransMVSNet.py:75-78."""
    new = proj[:, 0].clone()
    new[:, :3, :4] = torch.matmul(proj[:, 1, :3, :3], proj[:, 0, :3, :4])
    return new


def warp_grid(src_proj, ref_proj, depth_values, height, width):
    """Grid construction of homo_warping, models/module.py:294-316. Returns [B, D*H, W, 2]."""
    batch = depth_values.shape[0]
    num_depth = depth_values.shape[1]
    with torch.no_grad():
        proj = torch.matmul(src_proj, torch.inverse(ref_proj))
        rot = proj[:, :3, :3]
        trans = proj[:, :3, 3:4]
        y, x = torch.meshgrid([torch.arange(0, height, dtype=depth_values.dtype),
                               torch.arange(0, width, dtype=depth_values.dtype)], indexing="ij")
        y, x = y.contiguous().view(height * width), x.contiguous().view(height * width)
        xyz = torch.stack((x, y, torch.ones_like(x)))
        xyz = torch.unsqueeze(xyz, 0).repeat(batch, 1, 1)
        rot_xyz = torch.matmul(rot, xyz)
        rot_depth_xyz = rot_xyz.unsqueeze(2).repeat(1, 1, num_depth, 1) * depth_values.view(batch, 1, num_depth, -1)
        proj_xyz = rot_depth_xyz + trans.view(batch, 3, 1, 1)
        invalid = (proj_xyz[:, 2:3, :, :] < 1e-6).squeeze(1)
        proj_xy = proj_xyz[:, :2, :, :] / (proj_xyz[:, 2:3, :, :])
        px = proj_xy[:, 0, :, :] / ((width - 1) / 2) - 1
        px[invalid] = -99.
        py = proj_xy[:, 1, :, :] / ((height - 1) / 2) - 1
        py[invalid] = -99.
        grid = torch.stack((px, py), dim=3)
    return grid.view(batch, num_depth * height, width, 2)


def homo_warping(src_fea, src_proj, ref_proj, depth_values):
    """homo_warping, models/module.py:284-322 -> [B, C, D, H, W]."""
    b, c, h, w = src_fea.shape
    d = depth_values.shape[1]
    grid = warp_grid(src_proj, ref_proj, depth_values, h, w)
    out = F.grid_sample(src_fea, grid, mode="bilinear", padding_mode="zeros", align_corners=True)
    return out.view(b, c, d, h, w)


def pixelwise_net(sd, sim, p="DepthNet.pixel_wise_net.", training=False):
    """PixelwiseNet.forward, models/TransMVSNet.py:20-30 -> [B,1,H,W] (training: BN batch statistics)."""
    x = F.relu(_bn(F.conv3d(sim, sd[p + "conv0.conv.weight"]), sd, p + "conv0.bn.", training))
    x = F.relu(_bn(F.conv3d(x, sd[p + "conv1.conv.weight"]), sd, p + "conv1.bn.", training))
    x = F.conv3d(x, sd[p + "conv2.weight"], sd[p + "conv2.bias"]).squeeze(1)
    return torch.max(torch.sigmoid(x), dim=1, keepdim=True)[0]


def build_cost_volume(sd, features, proj_matrix, depth_values, view_weights=None, training=False):
    """Steps 1-2 of DepthNet.forward, models/TransMVSNet.py:58-93.

    Returns (similarity [B,1,D,H,W], view_weights [B,V,H,W] or None).
    """
    projs = torch.unbind(proj_matrix, 1)
    ref_fea, src_feas = features[0], features[1:]
    ref_proj, src_projs = projs[0], projs[1:]
    weights_out = [] if view_weights is None else None
    sim_sum = 0
    w_sum = 1e-5
    for i, (src_fea, src_proj) in enumerate(zip(src_feas, src_projs)):
        warped = homo_warping(src_fea, compose_proj(src_proj), compose_proj(ref_proj), depth_values)
        sim = (warped * ref_fea.unsqueeze(2)).mean(1, keepdim=True)
        if view_weights is None:
            vw = pixelwise_net(sd, sim, training=training)
            weights_out.append(vw)
        else:
            vw = view_weights[:, i:i + 1]
        sim_sum += sim * vw.unsqueeze(1)
        w_sum += vw.unsqueeze(1)
        del warped
    sim = sim_sum.div_(w_sum)
    return sim, (torch.cat(weights_out, dim=1) if weights_out is not None else None)


# ----------------------------------------------------------------------------- CostRegNet
def _conv3d_bn_relu(sd, p, x, stride, training=False):
    return F.relu(_bn(F.conv3d(x, sd[p + "conv.weight"], stride=stride, padding=1), sd, p + "bn.", training))


def _deconv3d_bn_relu(sd, p, x, training=False):
    y = F.conv_transpose3d(x, sd[p + "conv.weight"], stride=2, padding=1, output_padding=1)
    return F.relu(_bn(y, sd, p + "bn.", training))


def cost_reg_net(sd, p, x, training=False):
    """CostRegNet.forward, models/module.py:447-456 (Conv3d :135-141, Deconv3d :179-185); training=True
    is the module in train mode (BatchNorm3d batch statistics, running statistics updated)."""
    t = training
    conv0 = _conv3d_bn_relu(sd, p + "conv0.", x, 1, t)
    conv2 = _conv3d_bn_relu(sd, p + "conv2.", _conv3d_bn_relu(sd, p + "conv1.", conv0, 2, t), 1, t)
    conv4 = _conv3d_bn_relu(sd, p + "conv4.", _conv3d_bn_relu(sd, p + "conv3.", conv2, 2, t), 1, t)
    x = _conv3d_bn_relu(sd, p + "conv6.", _conv3d_bn_relu(sd, p + "conv5.", conv4, 2, t), 1, t)
    x = conv4 + _deconv3d_bn_relu(sd, p + "conv7.", x, t)
    x = conv2 + _deconv3d_bn_relu(sd, p + "conv9.", x, t)
    x = conv0 + _deconv3d_bn_relu(sd, p + "conv11.", x, t)
    return F.conv3d(x, sd[p + "prob.weight"], stride=1, padding=1)


# ----------------------------------------------------------------------------- regression
def depth_wta(p, depth_values):
    """depth_wta, models/module.py:474-482 (argmax = first max)."""
    idx = torch.argmax(p, dim=1, keepdim=True).type(torch.long)
    return torch.gather(depth_values, 1, idx).squeeze(1)


def softmax_regression(cost_reg, depth_values):
    """models/TransMVSNet.py:97-103."""
    prob = torch.exp(F.log_softmax(cost_reg.squeeze(1), dim=1))
    depth = depth_wta(prob, depth_values)
    conf = torch.max(prob, dim=1)[0]
    return prob, depth, conf


def depth_net(sd, features, proj_matrix, depth_values, stage_idx, view_weights=None, training=False):
    """DepthNet.forward, models/TransMVSNet.py:38-109 (returns dict, view_weights)."""
    sim, vw = build_cost_volume(sd, features, proj_matrix, depth_values, view_weights, training=training)
    cost = cost_reg_net(sd, f"cost_regularization.{stage_idx}.", sim, training=training)
    prob, depth, conf = softmax_regression(cost, depth_values)
    if training:
        conf = conf.detach()  # computed under torch.no_grad() (models/TransMVSNet.py:102-103)
    out = {"depth": depth, "photo_confidence": conf, "prob_volume": prob, "depth_values": depth_values}
    return out, (vw.detach() if vw is not None else None)


def get_depth_samples(cur_depth, ndepth, depth_inteval_pixel, shape):
    """get_depth_samples, models/module.py:606-634 (min/max_depth args unused there)."""
    if cur_depth.dim() == 2:
        dmin = cur_depth[:, 0]
        dmax = cur_depth[:, -1]
        new_interval = (dmax - dmin) / (ndepth - 1)
        s = dmin.unsqueeze(1) + (torch.arange(0, ndepth, dtype=cur_depth.dtype).reshape(1, -1) * new_interval.unsqueeze(1))
        return s.unsqueeze(-1).unsqueeze(-1).repeat(1, 1, shape[1], shape[2])
    dmin = cur_depth - ndepth / 2 * depth_inteval_pixel
    dmax = cur_depth + ndepth / 2 * depth_inteval_pixel
    new_interval = (dmax - dmin) / (ndepth - 1)
    return dmin.unsqueeze(1) + (torch.arange(0, ndepth, dtype=cur_depth.dtype).reshape(1, -1, 1, 1) * new_interval.unsqueeze(1))


def stage_hypotheses(depth, depth_values, stage_idx, img_hw, ndepths=NDEPTHS, ratios=DEPTH_RATIOS):
    """Stage glue, models/TransMVSNet.py:147-149,174-204: hypotheses [B, D, H/s, W/s]."""
    h, w = img_hw
    depth_min = float(depth_values[0, 0].numpy())
    depth_max = float(depth_values[0, -1].numpy())
    depth_interval = (depth_max - depth_min) / depth_values.size(1)
    if depth is not None:
        cur = F.interpolate(depth.detach().unsqueeze(1), [h, w], mode="bilinear",
                            align_corners=ALIGN_CORNERS_RANGE).squeeze(1)
    else:
        cur = depth_values
    samples = get_depth_samples(cur, ndepths[stage_idx], ratios[stage_idx] * depth_interval,
                                [depth_values.shape[0], h, w])
    s = STAGE_SCALES[stage_idx]
    return F.interpolate(samples.unsqueeze(1), [ndepths[stage_idx], h // s, w // s], mode="trilinear",
                         align_corners=ALIGN_CORNERS_RANGE).squeeze(1)


def forward_from_features(sd, features, proj_matrix, depth_values, img_hw, ndepths=NDEPTHS, ratios=DEPTH_RATIOS,
                          with_view_weights=False, training=False, pyramid=None, seed_depth=None):
    """TransMVSNet.forward after feature extraction, models/TransMVSNet.py:162-226 (training: the
    model in train mode -- BatchNorm batch statistics + running-statistic updates; autograd flows
    as in the reference: hypotheses and the next stage's depth detached, stage-1 view weights
    detached for stages 2/3).

    Test hooks: pyramid = a precomputed fmt_with_pathway(sd, features) (not recomputed);
    seed_depth = {"stage2": depth, "stage3": depth}: the previous stage's unclamped WTA depth [B,h,w]
    that stage's hypotheses are built from (TransMVSNet.py:174-213) in place of this run's own -- the
    reference cascade continued from another implementation's previous-stage depth."""
    feats = fmt_with_pathway(sd, features) if pyramid is None else pyramid
    outputs = {}
    depth = None
    view_weights = None
    for s in range(len(ndepths)):
        name = f"stage{s + 1}"
        if seed_depth is not None and name in seed_depth:
            depth = seed_depth[name]
        hyp = stage_hypotheses(depth, depth_values, s, img_hw, ndepths, ratios)
        if s > 0:
            view_weights = F.interpolate(view_weights, scale_factor=2, mode="nearest")
        out, vw = depth_net(sd, [f[name] for f in feats], proj_matrix[name], hyp, s, view_weights, training)
        if s == 0:
            view_weights = vw
            stage1_vw = vw
        idx = torch.argmax(out["prob_volume"], dim=1, keepdim=True).type(torch.long)
        depth = torch.gather(out["depth_values"], 1, idx).squeeze(1)
        out["depth"] = depth.clamp(*DEPTH_CLAMP)
        outputs[name] = out
        outputs.update(out)
    if with_view_weights:
        return outputs, stage1_vw
    return outputs


# ----------------------------------------------------------------------------- FeatureNet (context, not the hot path)
def deform_conv2d(x, offset, weight, bias, padding, mask):
    """torchvision.ops.deform_conv2d (torchvision 0.10.1, requirements.txt:13; call site
    models/dcn.py:71-80) restated: stride 1, dilation 1, one offset group. Offsets are
    interleaved (dy, dx) per tap; bilinear sampling with zeros outside; the modulated
    column is ``mask * bilinear(x, p + p_k + offset_k)``; then a GEMM with the weights.
    Parity of this third-party arithmetic is unpinned (no reference test holds it);
    at the reference's zero-initialised offsets (models/dcn.py:62-64) it is exact.
    """
    b, c, h, w = x.shape
    co, _, kh, kw = weight.shape
    ys = torch.arange(h, dtype=x.dtype).view(1, h, 1).expand(b, h, w)
    xs = torch.arange(w, dtype=x.dtype).view(1, 1, w).expand(b, h, w)
    flat = x.reshape(b, c, h * w)
    cols = []
    for i in range(kh):
        for j in range(kw):
            k = i * kw + j
            py = ys + float(i - padding) + offset[:, 2 * k]
            px = xs + float(j - padding) + offset[:, 2 * k + 1]
            inside = (py > -1) & (py < h) & (px > -1) & (px < w)
            y0 = torch.floor(py)
            x0 = torch.floor(px)
            ly, lx = py - y0, px - x0
            hy, hx = 1 - ly, 1 - lx
            y0i, x0i = y0.long(), x0.long()
            val = 0
            for dy, dx, wt in ((0, 0, hy * hx), (0, 1, hy * lx), (1, 0, ly * hx), (1, 1, ly * lx)):
                yy, xx = y0i + dy, x0i + dx
                ok = inside & (yy >= 0) & (yy <= h - 1) & (xx >= 0) & (xx <= w - 1)
                lin = (yy.clamp(0, h - 1) * w + xx.clamp(0, w - 1)).view(b, 1, h * w).expand(b, c, h * w)
                tap = torch.gather(flat, 2, lin).view(b, c, h, w) * ok.unsqueeze(1)
                val = val + wt.unsqueeze(1) * tap
            cols.append(mask[:, k:k + 1] * val)
    col = torch.stack(cols, dim=2).view(b, c * kh * kw, h * w)
    out = torch.matmul(weight.view(co, -1), col).view(b, co, h, w)
    if bias is not None:
        out = out + bias.view(1, -1, 1, 1)
    return out


def _dcn(sd, p, x):
    """DCN.forward, models/dcn.py:66-80."""
    out = F.conv2d(x, sd[p + "conv_offset_mask.weight"], sd[p + "conv_offset_mask.bias"], padding=1)
    o1, o2, mask = torch.chunk(out, 3, dim=1)
    offset = torch.cat((o1, o2), dim=1)
    mask = torch.sigmoid(mask)
    return deform_conv2d(x, offset, sd[p + "weight"], sd[p + "bias"], 1, mask)


def _conv2d_bn_relu(sd, p, x, stride, padding, training=False):
    """Conv2d block, models/module.py:49-56 (bn + relu)."""
    y = F.conv2d(x, sd[p + "conv.weight"], stride=stride, padding=padding)
    return F.relu(_bn(y, sd, p + "bn.", training))


def _out_head(sd, p, x, first_k, training=False, dcn=_dcn):
    """FeatureNet.out{1,2,3} Sequentials, models/module.py:362-395."""
    t = training
    x = _conv2d_bn_relu(sd, p + "0.", x, 1, 0 if first_k == 1 else 1, t)
    x = F.relu(_bn(dcn(sd, p + "1.", x), sd, p + "2.", t))
    x = F.relu(_bn(dcn(sd, p + "4.", x), sd, p + "5.", t))
    return dcn(sd, p + "7.", x)


def feature_net(sd, x, p="feature.", training=False, dcn=_dcn):
    """FeatureNet.forward, models/module.py:399-422 (training: BatchNorm2d batch statistics of this
    call's batch -- the reference calls FeatureNet once per view, models/TransMVSNet.py:151-153).
    dcn: the DCN block's function (a test may wrap _dcn in activation checkpointing: same values)."""
    t = training
    conv0 = _conv2d_bn_relu(sd, p + "conv0.1.", _conv2d_bn_relu(sd, p + "conv0.0.", x, 1, 1, t), 1, 1, t)
    c1 = _conv2d_bn_relu(sd, p + "conv1.0.", conv0, 2, 2, t)
    conv1 = _conv2d_bn_relu(sd, p + "conv1.2.", _conv2d_bn_relu(sd, p + "conv1.1.", c1, 1, 1, t), 1, 1, t)
    c2 = _conv2d_bn_relu(sd, p + "conv2.0.", conv1, 2, 2, t)
    conv2 = _conv2d_bn_relu(sd, p + "conv2.2.", _conv2d_bn_relu(sd, p + "conv2.1.", c2, 1, 1, t), 1, 1, t)
    out = {"stage1": _out_head(sd, p + "out1.", conv2, 1, t, dcn)}
    intra = F.interpolate(conv2, scale_factor=2.0, mode="nearest") + F.conv2d(conv1, sd[p + "inner1.weight"], sd[p + "inner1.bias"])
    out["stage2"] = _out_head(sd, p + "out2.", intra, 3, t, dcn)
    intra = F.interpolate(intra, scale_factor=2.0, mode="nearest") + F.conv2d(conv0, sd[p + "inner2.weight"], sd[p + "inner2.bias"])
    out["stage3"] = _out_head(sd, p + "out3.", intra, 3, t, dcn)
    return out


def forward(sd, imgs, proj_matrix, depth_values, training=False, **kw):
    """TransMVSNet.forward, models/TransMVSNet.py:141-226."""
    feats = [feature_net(sd, imgs[:, v], training=training) for v in range(imgs.size(1))]
    return forward_from_features(sd, feats, proj_matrix, depth_values, (imgs.shape[3], imgs.shape[4]),
                                 training=training, **kw)
