"""FeatureNet + DCN (models/module.py:343-422, models/dcn.py:43-80) -- SURVEY.md 8f, the #1 "next" row.

Every layer is a HIP kernel behind the C-ABI, NHWC end to end: the trunk's Conv+BN+ReLU blocks
and the stage-1 head's 1x1 (``tmvs_conv2d_bn_relu``, csrc/conv2d.hip), the FPN merges
(``tmvs_fpn_merge``), the stage-2/3 heads' 3x3 blocks (``tmvs_conv3x3_nhwc``), and each DCN -- its
conv_offset_mask conv AND the modulated deformable convolution (torchvision.ops.deform_conv2d,
torchvision 0.10.1, absent in this image) -- as ONE launch, ``tmvs_dcn_fused`` (csrc/featurenet.hip),
with the head's bias, BatchNorm and ReLU fused into its epilogue (models/module.py:362-395: DCN ->
BN -> ReLU -> DCN -> BN -> ReLU -> DCN); the offset/mask tensor never reaches HBM. The stage
outputs are NCHW, as the reference's. There is no CPU path. Module/parameter names are the
reference's, so checkpoints load strict=True.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import ops


class Conv2dBlock(nn.Module):
    """Conv2d + BN + ReLU block (models/module.py:24-61)."""

    def __init__(self, cin, cout, k, stride=1, padding=0):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride=stride, padding=padding, bias=False)
        self.bn = nn.BatchNorm2d(cout, momentum=0.1)
        self._packed = None
        self.register_load_state_dict_post_hook(lambda m, k: setattr(m, "_packed", None))

    def forward(self, x):
        raise RuntimeError("Conv2dBlock is a parameter container: use forward_native / forward_nhwc (HIP)")

    def forward_native(self, x, nchw_input=False):
        """This block as one HIP kernel (tmvs_conv2d_bn_relu): NHWC in (or the NCHW image), NHWC out."""
        bn, conv = self.bn, self.conv
        key = ("c2d", str(x.device), conv.weight._version, bn.weight._version, bn.bias._version,
               bn.running_mean._version, bn.running_var._version)
        if self._packed is None or self._packed[0] != key:
            a, s = ops.bn_fold(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps)
            self._packed = (key, ops.conv2d_pack(conv.weight).to(x.device),
                            (torch.from_numpy(a).to(x.device), torch.from_numpy(s).to(x.device)))
        return ops.conv2d_bn_relu(x, self._packed[1], conv.out_channels, conv.kernel_size[0], conv.stride[0],
                                  bn=self._packed[2], relu=True, nchw_input=nchw_input)

    def forward_nhwc(self, x_nhwc):
        """The heads' 3x3 32 -> 32 block on NHWC input as one HIP kernel (tmvs_conv3x3_nhwc) -> NHWC."""
        bn = self.bn
        key = ("dcnpk", str(x_nhwc.device), self.conv.weight._version, bn.weight._version, bn.bias._version,
               bn.running_mean._version, bn.running_var._version)
        if self._packed is None or self._packed[0] != key:
            a, s = ops.bn_fold(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps)
            self._packed = (key, ops.deform_conv2d_pack(self.conv.weight).to(x_nhwc.device),
                            (torch.from_numpy(a).to(x_nhwc.device), torch.from_numpy(s).to(x_nhwc.device)))
        return ops.conv3x3_nhwc(x_nhwc, self._packed[1], bn=self._packed[2], relu=True)[1]


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
        com = self.conv_offset_mask
        key = (str(device), self.weight._version, self.bias._version, com.weight._version, com.bias._version, bnv)
        if self._packed is None or self._packed[0] != key:
            w = ops.deform_conv2d_pack(self.weight).to(device)
            b = self.bias.detach().float().contiguous().to(device)
            wom = ops.deform_conv2d_pack(com.weight).to(device)
            bom = com.bias.detach().float().contiguous().to(device)
            fold = None
            if bn is not None:
                a, s = ops.bn_fold(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps)
                fold = (torch.from_numpy(a).to(device), torch.from_numpy(s).to(device))
            self._packed = (key, w, b, wom, bom, fold)
        return self._packed[1:]

    def forward(self, x_nhwc, bn=None, relu=False, want_nchw=True, want_nhwc=False):
        """DCN.forward (models/dcn.py:66-80) on x_nhwc [B,H,W,32]: conv_offset_mask, deform_conv2d, then
        the head's eval BatchNorm ``bn`` and ReLU if given -- one fused kernel. Returns (nchw, nhwc)."""
        if not x_nhwc.is_cuda:
            raise RuntimeError("FeatureNet DCN runs on the GPU only (tmvs_dcn_fused); no CPU fallback")
        w, b, wom, bom, fold = self._prepared(x_nhwc.device, bn)
        return ops.dcn_fused(x_nhwc.contiguous(), wom, bom, w, b, self.cout, bn=fold, relu=relu, want_nchw=want_nchw,
                             want_nhwc=want_nhwc)


def _head(cin, cmid, cout, first_k):
    return nn.Sequential(
        Conv2dBlock(cin, cmid, first_k, 1, 0 if first_k == 1 else 1),
        DCN(cmid, cmid), nn.BatchNorm2d(cmid), nn.ReLU(inplace=True),
        DCN(cmid, cmid), nn.BatchNorm2d(cmid), nn.ReLU(inplace=True),
        DCN(cmid, cout))


def _run_head(seq, x, x_nhwc=None):
    """out{1,2,3} Sequential (models/module.py:362-395) with BN + ReLU fused into the DCN kernels.
    With x_nhwc (stages 2/3) the first 3x3 block also runs natively."""
    if x_nhwc is not None:  # 3x3 first block (stages 2/3)
        xh = seq[0].forward_nhwc(x_nhwc)
    else:  # 1x1 first block (stage 1) on the NHWC trunk output
        xh = seq[0].forward_native(x)
    _, xh = seq[1](xh, bn=seq[2], relu=True, want_nchw=False, want_nhwc=True)
    _, xh = seq[4](xh, bn=seq[5], relu=True, want_nchw=False, want_nhwc=True)
    return seq[7](xh)[0]


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
        x = x.contiguous()
        if not x.is_cuda:
            raise RuntimeError("FeatureNet runs on the GPU only (HIP kernels); no CPU fallback")
        conv0 = self.conv0[1].forward_native(self.conv0[0].forward_native(x, nchw_input=True))  # NHWC from here on
        conv1 = conv0
        for blk in self.conv1:
            conv1 = blk.forward_native(conv1)
        conv2 = conv1
        for blk in self.conv2:
            conv2 = blk.forward_native(conv2)
        out = {"stage1": _run_head(self.out1, conv2)}
        # intra = interpolate(., 2, nearest) + inner(.) as one NHWC kernel (models/module.py:413, 417)
        intra = ops.fpn_merge(conv2, conv1, *self._inner(self.inner1, conv2.device))
        out["stage2"] = _run_head(self.out2, None, intra)
        intra = ops.fpn_merge(intra, conv0, *self._inner(self.inner2, conv2.device))
        out["stage3"] = _run_head(self.out3, None, intra)
        return out

    def _inner(self, conv, device):
        """inner{1,2} 1x1 conv weight [32, cl] and bias, cached per parameter version."""
        key = (id(conv), str(device), conv.weight._version, conv.bias._version)
        cache = self.__dict__.setdefault("_inner_cache", {})
        if cache.get(id(conv), (None,))[0] != key:
            w = conv.weight.detach().float().reshape(conv.out_channels, conv.in_channels).contiguous().to(device)
            cache[id(conv)] = (key, w, conv.bias.detach().float().contiguous().to(device))
        return cache[id(conv)][1:]
