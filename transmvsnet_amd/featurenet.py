"""FeatureNet + DCN (models/module.py:343-422, models/dcn.py:43-80) -- SURVEY.md 8f, the #1 "next" row.

The 3-scale trunk, the lateral 1x1 convs and each DCN's offset/mask conv run as PyTorch-ROCm
(MIOpen) convolutions. The modulated deformable convolution itself -- torchvision.ops.deform_conv2d
(torchvision 0.10.1, absent in this image) -- runs as the HIP kernel ``tmvs_deform_conv2d``
(csrc/featurenet.hip), with the head's bias, BatchNorm and ReLU fused into its epilogue
(models/module.py:362-395: DCN -> BN -> ReLU -> DCN -> BN -> ReLU -> DCN). There is no CPU path.
The module/parameter names are the reference's, so checkpoints load strict=True.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


class Conv2dBlock(nn.Module):
    """Conv2d + BN + ReLU block (models/module.py:24-61)."""

    def __init__(self, cin, cout, k, stride=1, padding=0):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride=stride, padding=padding, bias=False)
        self.bn = nn.BatchNorm2d(cout, momentum=0.1)

    def forward(self, x):
        return F.relu(self.bn(self.conv(x)))


class DCN(nn.Module):
    """DCNv2 (models/dcn.py:15-80): weight/bias + zero-initialised offset/mask conv."""

    def __init__(self, cin, cout, k=3, padding=1):
        super().__init__()
        self.padding = padding
        self.cout = cout
        self.weight = nn.Parameter(torch.empty(cout, cin, k, k))
        self.bias = nn.Parameter(torch.zeros(cout))
        std = 1.0 / math.sqrt(cin * k * k)
        nn.init.uniform_(self.weight, -std, std)
        self.conv_offset_mask = nn.Conv2d(cin, 3 * k * k, k, padding=padding, bias=True)
        nn.init.zeros_(self.conv_offset_mask.weight)
        nn.init.zeros_(self.conv_offset_mask.bias)
        self._packed = None
        self.register_load_state_dict_post_hook(lambda m, k: m.invalidate())

    def invalidate(self):
        self._packed = None

    def _prepared(self, device, bn):
        bnv = None if bn is None else (id(bn), bn.weight._version, bn.bias._version, bn.running_mean._version,
                                       bn.running_var._version)
        key = (str(device), self.weight._version, self.bias._version, bnv)
        if self._packed is None or self._packed[0] != key:
            w = ops.deform_conv2d_pack(self.weight).to(device)
            b = self.bias.detach().float().contiguous().to(device)
            fold = None
            if bn is not None:
                a, s = ops.bn_fold(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps)
                fold = (torch.from_numpy(a).to(device), torch.from_numpy(s).to(device))
            self._packed = (key, w, b, fold)
        return self._packed[1:]

    def forward(self, x, bn=None, relu=False, x_nhwc=None, want_nhwc=False):
        """deform_conv2d(x, offset, weight, bias, mask) (models/dcn.py:71-80), then the head's
        eval BatchNorm ``bn`` and ReLU if given (fused)."""
        if not x.is_cuda:
            raise RuntimeError("FeatureNet DCN runs on the GPU only (tmvs_deform_conv2d); no CPU fallback")
        om = self.conv_offset_mask(x).contiguous()
        if x_nhwc is None:
            x_nhwc = x.permute(0, 2, 3, 1).contiguous()
        w, b, fold = self._prepared(x.device, bn)
        return ops.deform_conv2d(x_nhwc, om, w, b, self.cout, bn=fold, relu=relu, want_nhwc=want_nhwc)


def _head(cin, cmid, cout, first_k):
    return nn.Sequential(
        Conv2dBlock(cin, cmid, first_k, 1, 0 if first_k == 1 else 1),
        DCN(cmid, cmid), nn.BatchNorm2d(cmid), nn.ReLU(inplace=True),
        DCN(cmid, cmid), nn.BatchNorm2d(cmid), nn.ReLU(inplace=True),
        DCN(cmid, cout))


def _run_head(seq, x):
    """out{1,2,3} Sequential (models/module.py:362-395) with BN + ReLU fused into the DCN kernels."""
    x = seq[0](x)
    x, xh = seq[1](x, bn=seq[2], relu=True, want_nhwc=True)
    x, xh = seq[4](x, bn=seq[5], relu=True, x_nhwc=xh, want_nhwc=True)
    return seq[7](x, x_nhwc=xh)


class FeatureNet(nn.Module):
    """3-scale feature pyramid (models/module.py:343-422)."""

    def __init__(self, base_channels=8):
        super().__init__()
        b = base_channels
        self.conv0 = nn.Sequential(Conv2dBlock(3, b, 3, 1, 1), Conv2dBlock(b, b, 3, 1, 1))
        self.conv1 = nn.Sequential(Conv2dBlock(b, 2 * b, 5, 2, 2), Conv2dBlock(2 * b, 2 * b, 3, 1, 1),
                                   Conv2dBlock(2 * b, 2 * b, 3, 1, 1))
        self.conv2 = nn.Sequential(Conv2dBlock(2 * b, 4 * b, 5, 2, 2), Conv2dBlock(4 * b, 4 * b, 3, 1, 1),
                                   Conv2dBlock(4 * b, 4 * b, 3, 1, 1))
        self.out1 = _head(4 * b, 4 * b, 4 * b, 1)
        self.inner1 = nn.Conv2d(2 * b, 4 * b, 1, bias=True)
        self.inner2 = nn.Conv2d(b, 4 * b, 1, bias=True)
        self.out2 = _head(4 * b, 4 * b, 2 * b, 3)
        self.out3 = _head(4 * b, 4 * b, b, 3)

    def forward(self, x):
        """x [B,3,H,W] -> {stage1: [B,32,H/4,W/4], stage2: [B,16,H/2,W/2], stage3: [B,8,H,W]}.
        Views may be batched on B (eval BatchNorm is per sample)."""
        conv0 = self.conv0(x)
        conv1 = self.conv1(conv0)
        conv2 = self.conv2(conv1)
        out = {"stage1": _run_head(self.out1, conv2)}
        intra = F.interpolate(conv2, scale_factor=2.0, mode="nearest") + self.inner1(conv1)
        out["stage2"] = _run_head(self.out2, intra)
        intra = F.interpolate(intra, scale_factor=2.0, mode="nearest") + self.inner2(conv0)
        out["stage3"] = _run_head(self.out3, intra)
        return out
