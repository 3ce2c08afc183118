"""TransMVSNet drop-in (models/TransMVSNet.py:112-226) over the MI355X HIP hot path.

``TransMVSNet`` has the reference's constructor, ``forward(imgs, proj_matrix, depth_values)``
signature, output dict and state_dict key layout (465 keys; checkpoints load strict=True).
Its submodules are parameter containers with the reference names; the depth-inference hot
path -- FMT linear attention, the FMT pathway, stage glue, the fused warp + correlation +
view-aggregation cost volume, CostRegNet and softmax/WTA -- runs as hand-written HIP kernels
through the C-ABI (include/transmvs.h). Weights are re-laid-out once per load_state_dict into
the kernels' packed formats (BN folded exactly as the reference CPU kernel folds it), and
re-packed whenever a parameter or buffer is replaced or updated in place. FeatureNet (SURVEY.md
8f rank 1) runs natively too (featurenet.py: trunk conv, FPN merge, fused DCN kernels).
Inference only: BatchNorm is folded with running statistics, so forward() refuses train mode.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch
import torch.nn as nn

from . import _lib, ops
from .featurenet import FeatureNet

NDEPTHS = (48, 32, 8)
RATIOS = (4.0, 1.0, 0.5)
STAGE_SCALES = (4, 2, 1)
DEPTH_CLAMP = (425.0, 935.0)
FMT_LAYERS = ("self", "cross") * 4

# Generation of parameter/buffer (re)registrations anywhere: `module.weight = Parameter(...)`,
# `load_state_dict(assign=True)` and buffer reassignment all go through register_parameter /
# register_buffer, so a changed generation means TransMVSNet._tracked may hold replaced tensors.
_REGISTRATION_GEN = [0]


def _bump_registration(*_):
    _REGISTRATION_GEN[0] += 1


nn.modules.module.register_module_parameter_registration_hook(_bump_registration)
nn.modules.module.register_module_buffer_registration_hook(_bump_registration)


# ----------------------------------------------------------------- parameter containers
class _AttentionLayer(nn.Module):
    """AttentionLayer (models/FMT.py:40-54) parameters."""

    def __init__(self, d=32):
        super().__init__()
        self.query_projection = nn.Linear(d, d)
        self.key_projection = nn.Linear(d, d)
        self.value_projection = nn.Linear(d, d)
        self.out_projection = nn.Linear(d, d)


class EncoderLayer(nn.Module):
    """EncoderLayer (models/FMT.py:78-94) parameters; forward runs in fmt.hip."""

    def __init__(self, d=32):
        super().__init__()
        self.attention = _AttentionLayer(d)
        self.linear1 = nn.Linear(d, 2 * d)
        self.linear2 = nn.Linear(2 * d, d)
        self.norm1 = nn.LayerNorm(d)
        self.norm2 = nn.LayerNorm(d)

    def packed(self):
        a = self.attention
        parts = [a.query_projection.weight, a.query_projection.bias, a.key_projection.weight.t(),
                 a.key_projection.bias, a.value_projection.weight.t(), a.value_projection.bias,
                 a.out_projection.weight, a.out_projection.bias, self.linear1.weight, self.linear1.bias,
                 self.linear2.weight.t(), self.linear2.bias, self.norm1.weight, self.norm1.bias, self.norm2.weight,
                 self.norm2.bias]
        flat = torch.cat([p.detach().float().contiguous().reshape(-1) for p in parts])
        assert flat.numel() == _lib.ENC_NPARAMS
        return flat


class FMT(nn.Module):
    """FMT (models/FMT.py:114-129): 8 layers, self/cross alternating; sine PE (not persistent)."""

    def __init__(self, d_model=32, nhead=8):
        super().__init__()
        self.d_model = d_model
        self.nhead = nhead
        self.layer_names = list(FMT_LAYERS)
        self.layers = nn.ModuleList([EncoderLayer(d_model) for _ in FMT_LAYERS])


class FMTWithPathway(nn.Module):
    """FMT_with_pathway (models/FMT.py:183-199) parameters."""

    def __init__(self, base_channels=8):
        super().__init__()
        b = base_channels
        self.FMT = FMT(4 * b, 8)
        self.dim_reduction_1 = nn.Conv2d(4 * b, 2 * b, 1, bias=False)
        self.dim_reduction_2 = nn.Conv2d(2 * b, b, 1, bias=False)
        self.smooth_1 = nn.Conv2d(2 * b, 2 * b, 3, padding=1, bias=False)
        self.smooth_2 = nn.Conv2d(b, b, 3, padding=1, bias=False)


class _ConvBn3d(nn.Module):
    def __init__(self, cin, cout, k=3, stride=1, padding=1, transposed=False):
        super().__init__()
        if transposed:
            self.conv = nn.ConvTranspose3d(cin, cout, k, stride=2, padding=1, output_padding=1, bias=False)
        else:
            self.conv = nn.Conv3d(cin, cout, k, stride=stride, padding=padding, bias=False)
        self.bn = nn.BatchNorm3d(cout, momentum=0.1)


class CostRegNet(nn.Module):
    """CostRegNet (models/module.py:425-445) parameters; forward runs in costreg.hip."""

    def __init__(self, in_channels=1, base_channels=8):
        super().__init__()
        b = base_channels
        self.base_channels = b
        self.conv0 = _ConvBn3d(in_channels, b)
        self.conv1 = _ConvBn3d(b, 2 * b, stride=2)
        self.conv2 = _ConvBn3d(2 * b, 2 * b)
        self.conv3 = _ConvBn3d(2 * b, 4 * b, stride=2)
        self.conv4 = _ConvBn3d(4 * b, 4 * b)
        self.conv5 = _ConvBn3d(4 * b, 8 * b, stride=2)
        self.conv6 = _ConvBn3d(8 * b, 8 * b)
        self.conv7 = _ConvBn3d(8 * b, 4 * b, transposed=True)
        self.conv9 = _ConvBn3d(4 * b, 2 * b, transposed=True)
        self.conv11 = _ConvBn3d(2 * b, b, transposed=True)
        self.prob = nn.Conv3d(b, 1, 3, stride=1, padding=1, bias=False)

    def packed(self, device):
        """Device tensors in TmvsCostRegWeights order (include/transmvs.h)."""
        ws, als, shs = [], [], []

        def conv_w(w):  # [Co][Ci][3,3,3] -> [27][Co][Ci]
            co, ci = w.shape[:2]
            return w.detach().float().reshape(co, ci, 27).permute(2, 0, 1).contiguous()

        def deconv_w(w):  # [Ci][Co][3,3,3] -> [27][Co][Ci]
            ci, co = w.shape[:2]
            return w.detach().float().reshape(ci, co, 27).permute(2, 1, 0).contiguous()

        names = ["conv0", "conv1", "conv2", "conv3", "conv4", "conv5", "conv6", "conv7", "conv9", "conv11"]
        for i, n in enumerate(names):
            blk = getattr(self, n)
            w = blk.conv.weight
            if i < 7:
                ws.append(conv_w(w))
            else:
                ws.append(deconv_w(w))
            a, s = ops.bn_fold(blk.bn.weight, blk.bn.bias, blk.bn.running_mean, blk.bn.running_var, blk.bn.eps)
            als.append(torch.from_numpy(a))
            shs.append(torch.from_numpy(s))
        # prob [1][C][kd][kh][kw] -> per kh: 24 {kd1, kd2} pairs in (kw, c) order, then 24 kd0 in (kw, c) order
        pw = self.prob.weight.detach().float().reshape(self.base_channels, 3, 3, 3)
        pairs = pw[:, 1:3].permute(2, 3, 0, 1).reshape(3, -1)
        single = pw[:, 0].permute(1, 2, 0).reshape(3, -1)
        ws.append(torch.cat([pairs, single], 1).contiguous())
        ws = [t.to(device) for t in ws]
        als = [t.to(device) for t in als]
        shs = [t.to(device) for t in shs]
        st = _lib.CostRegWeights()
        for i, t in enumerate(ws):
            st.w[i] = t.data_ptr()
        for i in range(10):
            st.alpha[i] = als[i].data_ptr()
            st.shift[i] = shs[i].data_ptr()
        st.base_ch = self.base_channels
        return st, ws + als + shs


class _ConvBnReLU3D(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv = nn.Conv3d(cin, cout, 1, stride=1, padding=0, bias=False)
        self.bn = nn.BatchNorm3d(cout)


class PixelwiseNet(nn.Module):
    """PixelwiseNet (models/TransMVSNet.py:10-18) parameters."""

    def __init__(self):
        super().__init__()
        self.conv0 = _ConvBnReLU3D(1, 16)
        self.conv1 = _ConvBnReLU3D(16, 8)
        self.conv2 = nn.Conv3d(8, 1, 1, stride=1, padding=0)

    def packed(self):
        a0, s0 = ops.bn_fold(self.conv0.bn.weight, self.conv0.bn.bias, self.conv0.bn.running_mean,
                             self.conv0.bn.running_var, self.conv0.bn.eps)
        a1, s1 = ops.bn_fold(self.conv1.bn.weight, self.conv1.bn.bias, self.conv1.bn.running_mean,
                             self.conv1.bn.running_var, self.conv1.bn.eps)
        f = lambda t: t.detach().float().cpu().reshape(-1).numpy()  # noqa: E731
        out = np.concatenate([f(self.conv0.conv.weight), a0, s0, f(self.conv1.conv.weight), a1, s1,
                              f(self.conv2.weight), f(self.conv2.bias)]).astype(np.float32)
        assert out.size == _lib.PW_NPARAMS
        return out


class DepthNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.pixel_wise_net = PixelwiseNet()


def position_encoding_sine(d_model, h, w, max_shape=(600, 600)):
    """PositionEncodingSine buffer slice (models/position_encoding.py:28-60), same fp32 ops."""
    pe = torch.zeros((d_model, *max_shape))
    y_pos = torch.ones(max_shape).cumsum(0).float().unsqueeze(0)
    x_pos = torch.ones(max_shape).cumsum(1).float().unsqueeze(0)
    div = torch.exp(torch.arange(0, d_model // 2, 2).float() * (-math.log(10000.0) / (d_model // 2)))[:, None, None]
    pe[0::4] = torch.sin(x_pos * div)
    pe[1::4] = torch.cos(x_pos * div)
    pe[2::4] = torch.sin(y_pos * div)
    pe[3::4] = torch.cos(y_pos * div)
    return pe[:, :h, :w].contiguous()


# ----------------------------------------------------------------- the model
class TransMVSNet(nn.Module):
    def __init__(self, ndepths=(48, 32, 8), depth_interals_ratio=(4.0, 1.0, 0.5), cr_base_chs=(8, 8, 8)):
        super().__init__()
        assert len(ndepths) == len(depth_interals_ratio)
        self.ndepths = list(ndepths)
        self.depth_interals_ratio = list(depth_interals_ratio)
        self.cr_base_chs = list(cr_base_chs)
        self.num_stage = len(ndepths)
        self.stage_scales = {"stage1": 4.0, "stage2": 2.0, "stage3": 1.0}
        self.feature = FeatureNet(base_channels=8)
        self.FMT_with_pathway = FMTWithPathway()
        self.cost_regularization = nn.ModuleList([CostRegNet(1, self.cr_base_chs[i]) for i in range(self.num_stage)])
        self.DepthNet = DepthNet()
        self._prep = None
        self._tracked = None
        self._tracked_gen = -1
        self._pe = {}
        self.decomposed = False  # True: one C-ABI call per op (instrumentation); False: native stage calls
        # the FMT pathway (stage-2/3 features) depends only on the FMT output: run it on a side
        # stream, concurrently with stage 1 (whose small CostRegNet grids leave the GPU idle)
        self.overlap_pathway = True
        # priority of that side stream (torch.cuda.Stream: lower = higher priority; 0 = default)
        self.side_priority = 0
        # the FMT's reference-view chain on that side stream, concurrent with the source views (bitwise the same)
        self.split_fmt = os.environ.get("TMVS_SPLIT_FMT", "1") != "0"  # (env: A/B switch)
        self.fmt_side_priority = int(os.environ.get("TMVS_FMT_SIDE_PRIO", "0"))
        # where the pathway forks: "fmt" = right after the FMT (measured 298.5 vs 297.8 depth maps/s for "warp" =
        # once stage 1's cost volume is queued, and 295.0 on the main stream; profiles/r22/stream_layout_ab.txt,
        # fork_join2_ab.txt, fork_late_ab.txt)
        self.pathway_fork = os.environ.get("TMVS_PATHWAY_FORK", "fmt")
        self.one_side_stream = os.environ.get("TMVS_ONE_SIDE", "0") == "1"  # FMT and pathway on one side stream (A/B)
        # stage 2 waits only for the pathway's stage-2 output, stage 3 for its stage-3 output (A/B)
        # (profiles/r22/batch2_ab.txt: 295.9 vs 295.3 depth maps/s in three alternations)
        self.pathway_join2 = os.environ.get("TMVS_PW_JOIN2", "1") == "1"
        # rounding of homo_warping's rot·(x, y, 1) to reproduce: 'auto' = the host torch's
        # (ops.host_rot_order), or 'fma' / 'plain' to pin it (fixtures made on another machine)
        self.warp_rot_order = "auto"
        self._side = {}
        # B > 1: one stream per sample (sample 0 on the caller's stream), see _forward_features
        self.batch_streams = True
        self._sample_streams = {}
        self.register_load_state_dict_post_hook(lambda m, k: m.invalidate())

    def _sample_stream(self, dev, i):
        key = (dev, i)
        if key not in self._sample_streams:
            self._sample_streams[key] = torch.cuda.Stream(dev)
        return self._sample_streams[key]

    def _apply(self, fn, *a, **kw):  # .to() / .cuda() / .float() replace tensors: re-track them
        self._tracked = None
        self._prep = None
        return super()._apply(fn, *a, **kw)

    def invalidate(self):
        """Drop packed kernel weights (after any in-place parameter change)."""
        self._prep = None
        self._tracked = None

    def _param_key(self):
        """Identity + in-place version of every parameter/buffer the packed weights derive from:
        an optimizer step or a .copy_() bumps a version, a `.data` reassignment changes a data_ptr,
        and replacing a Parameter/buffer object re-registers it (global hook above), which
        rebuilds the tracked list (walking the module tree costs ~0.7 ms, so it is cached)."""
        ts = self._tracked
        if ts is None or self._tracked_gen != _REGISTRATION_GEN[0]:
            self._tracked_gen = _REGISTRATION_GEN[0]
            ts = self._tracked = [t for t in list(self.parameters()) + list(self.buffers())]
        return (len(ts), sum(t._version for t in ts), hash(tuple(t.data_ptr() for t in ts)))

    # --------------------------------------------------------- weight preparation
    def _prepared(self, device):
        key = self._param_key()
        if self._prep is not None and self._prep["device"] == device and self._prep["key"] == key:
            return self._prep
        self._prep = None
        fp = self.FMT_with_pathway
        enc = [layer.packed().to(device) for layer in fp.FMT.layers]
        cr = [c.packed(device) for c in self.cost_regularization]
        self._prep = {
            "device": device,
            "key": key,
            "enc": enc,
            "red1": fp.dim_reduction_1.weight.detach().float().reshape(16, 32).t().contiguous().to(device),
            "red2": fp.dim_reduction_2.weight.detach().float().reshape(8, 16).t().contiguous().to(device),
            "sm1": fp.smooth_1.weight.detach().float().permute(1, 2, 3, 0).contiguous().to(device),
            "sm2": fp.smooth_2.weight.detach().float().permute(1, 2, 3, 0).contiguous().to(device),
            "cr": cr,
            "pw": self.DepthNet.pixel_wise_net.packed(),
        }
        return self._prep

    def _pe_slice(self, h, w, device):
        key = (h, w, str(device))
        if key not in self._pe:
            self._pe[key] = position_encoding_sine(32, h, w).to(device)
        return self._pe[key]

    # --------------------------------------------------------- forward
    def forward(self, imgs, proj_matrix, depth_values):
        """models/TransMVSNet.py:141-226. FeatureNet runs once over all B*N views (the reference
        loops over views, :151-153; eval BatchNorm is per sample, so batching is exact). In train
        mode (model.train()) the whole forward runs on the HIP training kernels with autograd
        (transmvsnet_amd.train.forward_train): BatchNorm batch statistics, running statistics
        updated, gradients to every parameter through loss.backward()."""
        if self.training:
            from .train import forward_train
            self._prep = None  # parameters are about to change: drop the packed inference weights
            return forward_train(self, imgs, proj_matrix, depth_values)
        self._check_eval()
        b, n = imgs.shape[:2]
        with torch.cuda.device(imgs.device):
            f = self.feature(imgs.reshape(b * n, *imgs.shape[2:]))
        feats = {k: v.reshape(b, n, *v.shape[1:]) for k, v in f.items()}
        return self.forward_features(feats, proj_matrix, depth_values, (imgs.shape[3], imgs.shape[4]))

    def _check_eval(self):
        if self.training:
            raise RuntimeError("transmvsnet_amd.TransMVSNet.forward_features runs inference only (BatchNorm folded "
                               "with running statistics); call .eval() first, or forward() for training")

    @staticmethod
    def stack_features(features):
        """list of per-view {stage: [B,C,h,w]} -> {stage: [B,N,C,h,w]} contiguous."""
        if isinstance(features, dict):
            return {k: v.contiguous() for k, v in features.items()}
        return {k: torch.stack([f[k] for f in features], 1).contiguous() for k in ("stage1", "stage2", "stage3")}

    def forward_features(self, features, proj_matrix, depth_values, img_hw, return_view_weights=False,
                         view_shard=None):
        """Hot path after feature extraction (models/TransMVSNet.py:162-226).

        features: per-view list of FeatureNet dicts, or {stage: [B,N,C,h,w]} stacked.
        view_shard: optional transmvsnet_amd.distributed.ViewShard (source views split over ranks).
        """
        self._check_eval()
        feats = self.stack_features(features)
        if view_shard is not None:  # reference view + this rank's source views only
            feats = view_shard.select_features(feats)
        dev = feats["stage1"].device
        if not feats["stage1"].is_cuda:
            raise RuntimeError("TransMVSNet (HIP) needs GPU features; the HIP path has no CPU fallback")
        with torch.cuda.device(dev):  # kernels + current stream of the features' device
            return self._forward_features(feats, proj_matrix, depth_values, img_hw, return_view_weights,
                                          view_shard, dev)

    def _forward_features(self, feats, proj_matrix, depth_values, img_hw, return_view_weights, view_shard, dev):
        prep = self._prepared(dev)
        dv = depth_values.to(dev, torch.float32).contiguous()
        rows = {k: ops.proj_rows(proj_matrix[k]) for k in ("stage1", "stage2", "stage3")}
        if view_shard is not None:
            rows = {k: view_shard.select_rows(r) for k, r in rows.items()}
        b = feats["stage1"].shape[0]
        per = []
        vws = []
        # stage 1 samples each sample's own depth range; the stage-2/3 hypothesis interval comes
        # from depth_values[0] for every sample (models/TransMVSNet.py:146-148). Samples are independent:
        # with B > 1 each runs on its own stream (sample 0 on the caller's), so one sample's small
        # coarse-level grids overlap another's kernels; the caller's stream then waits for all of them.
        # Inside a HIP-graph capture the fork/join is captured too: each sample stream joins the capture by
        # waiting on an event of the capturing stream and is joined back before the capture ends; only the
        # caller's stream forks the FMT pathway's side stream (one fork level, _forward_one). (Round 5 turned
        # this off after a segfault at capture end; round 6 located it -- a two-level fork, the sample stream's
        # own pathway side stream, crashes hipStreamEndCapture -- DESIGN.md 7, tests/test_gpu_batch.py.)
        concurrent = b > 1 and self.batch_streams and view_shard is None and not self.decomposed
        main = torch.cuda.current_stream(dev)
        if concurrent:
            start = torch.cuda.Event()
            start.record(main)
        done = []
        for i in range(b):
            st = self._sample_stream(dev, i) if concurrent and i > 0 else main
            if st is not main:
                st.wait_event(start)
            with torch.cuda.stream(st):
                o, vw = self._forward_one({k: v[i] for k, v in feats.items()}, {k: r[i:i + 1] for k, r in rows.items()},
                                          dv[i:i + 1], dv[0:1], img_hw, prep, view_shard,
                                          slot=i if st is not main else 0, solo=not concurrent)
            if st is not main:
                ev = torch.cuda.Event()
                ev.record(st)
                done.append(ev)
                if not torch.cuda.is_current_stream_capturing():  # allocator: consumed on the caller's stream
                    for t in list(o[f"stage{s + 1}"][k] for s in range(self.num_stage) for k in o[f"stage{s + 1}"]) + [vw]:
                        if t is not None:
                            t.record_stream(main)
                    for t in feats.values():
                        t.record_stream(st)
            per.append(o)
            vws.append(vw)
        for ev in done:
            main.wait_event(ev)
        outputs = {}
        for s in range(self.num_stage):
            name = f"stage{s + 1}"
            if b == 1:
                outputs[name] = per[0][name]
            else:
                outputs[name] = {k: torch.cat([p[name][k] for p in per], 0) for k in per[0][name]}
            outputs.update(outputs[name])
        if return_view_weights:
            return outputs, (vws[0] if b == 1 else torch.cat(vws, 0))
        return outputs

    def _side_stream(self, dev, slot, role="pathway"):
        if self.one_side_stream:
            role = "pathway"
        key = (dev, slot, role)  # one side stream per sample stream (B > 1 runs samples concurrently) and role
        side = self._side.get(key)
        if side is None:
            prio = self.side_priority if role == "pathway" else self.fmt_side_priority
            side = self._side[key] = torch.cuda.Stream(dev, priority=prio)
        return side

    def _fmt(self, s1, prep, slot=0, solo=True):
        """FMT_with_pathway stage-1 part (models/FMT.py:212-226) -> tokens [N, h1*w1, 32].

        With split_fmt the reference view's chain runs on the side stream next to the source views
        (tmvs_fmt_forward_split, bitwise the same tokens); like the pathway, only from the caller's stream,
        and only when no other sample runs concurrently (solo): beside a second sample the extra fork measured
        slower (B = 2 on two streams 295.7 vs 303.6 depth maps/s, profiles/r22/batch2_ab.txt).
        """
        n, c, h1, w1 = s1.shape
        split = self.split_fmt and not self.decomposed and slot == 0 and solo
        side = self._side_stream(s1.device, slot, "fmt") if split else None
        return ops.fmt_forward(s1, self._pe_slice(h1, w1, s1.device), prep["enc"], side_stream=side)

    def _forward_one(self, f, rows, dv, dv0, img_hw, prep, view_shard, slot=0, solo=True):
        s1, s2, s3 = f["stage1"], f["stage2"], f["stage3"]
        n, _, h1, w1 = s1.shape
        tokens = self._fmt(s1, prep, slot, solo)
        st1 = tokens.view(n, h1, w1, 32)
        # the pathway's side stream forks only from the caller's stream (slot 0): a sample on its own stream
        # (slot > 0, B > 1) runs the pathway in line, so no stream forks from an already-forked stream -- a
        # HIP-graph capture of such a two-level fork (sample stream -> its side stream) segfaulted inside
        # hipStreamEndCapture on the box (r20a); the samples themselves still overlap each other
        overlap = self.overlap_pathway and not self.decomposed and slot == 0
        lateral = {}

        def pathway(side=None):
            lateral["st2"] = ops.fmt_pathway(st1, s2, prep["red1"], prep["sm1"])
            if side is not None:  # stage 2 needs only st2: it waits for this event, stage 3 for "done"
                lateral["done2"] = torch.cuda.Event()
                lateral["done2"].record(side)
            lateral["st3"] = ops.fmt_pathway(lateral["st2"], s3, prep["red2"], prep["sm2"])

        def pathway_side():
            """Launch the pathway on a side stream (right after the FMT, or once stage 1's cost volume is
            queued: pathway_fork), so it runs beside stage 1 (whose 1/16-resolution grids leave CUs idle)."""
            main = torch.cuda.current_stream(s1.device)
            side = self._side_stream(s1.device, slot)
            ready = torch.cuda.Event()
            ready.record(main)
            side.wait_event(ready)
            with torch.cuda.stream(side):
                pathway(side if self.pathway_join2 else None)
            done = torch.cuda.Event()
            done.record(side)
            # allocator bookkeeping: st2/st3 are consumed on the main stream, st1/s2/s3 read on side
            # (inside a HIP-graph capture the graph's private pool keeps every block alive instead)
            if not torch.cuda.is_current_stream_capturing():
                lateral["st2"].record_stream(main)
                lateral["st3"].record_stream(main)
                for t in (st1, s2, s3):
                    t.record_stream(side)
            lateral["done"] = done

        if not overlap:
            pathway()
        elif self.pathway_fork == "fmt":
            pathway_side()
        outputs = {}
        depth_raw = None
        view_w = None
        joined = not overlap  # the pathway's side stream joined back (a capture needs it before it ends)
        for s in range(self.num_stage):
            name = f"stage{s + 1}"
            if overlap and s == 1 and "done2" in lateral:
                torch.cuda.current_stream(s1.device).wait_event(lateral["done2"])
            elif overlap and s in (1, 2) and not joined:
                torch.cuda.current_stream(s1.device).wait_event(lateral["done"])
                joined = True
            fs = (st1, lateral.get("st2"), lateral.get("st3"))[s]
            if view_shard is None and not self.decomposed and s > 0:
                out, depth_raw = ops.depth_stage(dv0, depth_raw, fs, self.ndepths[s], self.depth_interals_ratio[s],
                                                 img_hw, STAGE_SCALES[s], rows[name][0], None, view_w, s,
                                                 prep["cr"][s][0], DEPTH_CLAMP, rot_order=self.warp_rot_order)
            else:  # per-op path: stage 1 (pathway launched between its cost volume and CostRegNet),
                # view-sharded mode, or per-kernel instrumentation -- the same kernels
                hyp = ops.stage_hypotheses(dv if s == 0 else dv0, depth_raw, self.ndepths[s], self.depth_interals_ratio[s], img_hw,
                                           STAGE_SCALES[s])
                if view_shard is not None:
                    sim, vw_new = view_shard.cost_volume(fs, rows[name], hyp, s, view_w, prep["pw"],
                                                         rot_order=self.warp_rot_order)
                elif s == 0:
                    sim, _, vw_new = ops.warp_corr(fs[0:1], fs[1:].unsqueeze(0), rows[name], hyp, pw_params=prep["pw"],
                                                   rot_order=self.warp_rot_order)
                else:
                    sim, _, _ = ops.warp_corr(fs[0:1], fs[1:].unsqueeze(0), rows[name], hyp, view_w_in=view_w,
                                              vw_shift=s, rot_order=self.warp_rot_order)
                if s == 0:
                    view_w = vw_new
                    if overlap and self.pathway_fork != "fmt":
                        pathway_side()
                prob, depth, depth_raw, conf = ops.costregnet_wta(sim, prep["cr"][s][0], hyp, DEPTH_CLAMP)
                out = {"depth": depth, "photo_confidence": conf, "prob_volume": prob, "depth_values": hyp}
            outputs[name] = out
        if not joined:  # fewer than 3 stages: the side stream still joins back
            torch.cuda.current_stream(s1.device).wait_event(lateral["done"])
        return outputs, view_w
