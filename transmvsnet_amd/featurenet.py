"""FeatureNet + DCN (models/module.py:343-422, models/dcn.py:43-80) -- OUTSIDE the hot path.

SURVEY.md section 8f ranks this the #1 "next" row (80 % of the FLOPs of a full forward, but
not named by the north star). Until its HIP kernels land it runs on the GPU through
PyTorch-ROCm (MIOpen convolutions) with a torch formulation of the modulated deformable
convolution (torchvision.ops.deform_conv2d, torchvision 0.10.1 -- absent in this image).
The module/parameter names are the reference's, so checkpoints load strict=True.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class Conv2dBlock(nn.Module):
    """Conv2d + BN + ReLU block (models/module.py:24-61)."""

    def __init__(self, cin, cout, k, stride=1, padding=0):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride=stride, padding=padding, bias=False)
        self.bn = nn.BatchNorm2d(cout, momentum=0.1)

    def forward(self, x):
        return F.relu(self.bn(self.conv(x)))


def deform_conv2d(x, offset, weight, bias, padding, mask):
    """Modulated deformable conv, stride 1 / dilation 1 / one offset group (torchvision layout:
    channel 2k = dy, 2k+1 = dx of tap k; bilinear, zeros outside)."""
    b, c, h, w = x.shape
    co, _, kh, kw = weight.shape
    ys = torch.arange(h, dtype=x.dtype, device=x.device).view(1, h, 1).expand(b, h, w)
    xs = torch.arange(w, dtype=x.dtype, device=x.device).view(1, 1, w).expand(b, h, w)
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
    return out if bias is None else out + bias.view(1, -1, 1, 1)


class DCN(nn.Module):
    """DCNv2 (models/dcn.py:15-80): weight/bias + zero-initialised offset/mask conv."""

    def __init__(self, cin, cout, k=3, padding=1):
        super().__init__()
        self.padding = padding
        self.weight = nn.Parameter(torch.empty(cout, cin, k, k))
        self.bias = nn.Parameter(torch.zeros(cout))
        std = 1.0 / math.sqrt(cin * k * k)
        nn.init.uniform_(self.weight, -std, std)
        self.conv_offset_mask = nn.Conv2d(cin, 3 * k * k, k, padding=padding, bias=True)
        nn.init.zeros_(self.conv_offset_mask.weight)
        nn.init.zeros_(self.conv_offset_mask.bias)

    def forward(self, x):
        o1, o2, m = torch.chunk(self.conv_offset_mask(x), 3, dim=1)
        return deform_conv2d(x, torch.cat((o1, o2), 1), self.weight, self.bias, self.padding, torch.sigmoid(m))


def _head(cin, cmid, cout, first_k):
    return nn.Sequential(
        Conv2dBlock(cin, cmid, first_k, 1, 0 if first_k == 1 else 1),
        DCN(cmid, cmid), nn.BatchNorm2d(cmid), nn.ReLU(inplace=True),
        DCN(cmid, cmid), nn.BatchNorm2d(cmid), nn.ReLU(inplace=True),
        DCN(cmid, cout))


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
        conv0 = self.conv0(x)
        conv1 = self.conv1(conv0)
        conv2 = self.conv2(conv1)
        out = {"stage1": self.out1(conv2)}
        intra = F.interpolate(conv2, scale_factor=2.0, mode="nearest") + self.inner1(conv1)
        out["stage2"] = self.out2(intra)
        intra = F.interpolate(intra, scale_factor=2.0, mode="nearest") + self.inner2(conv0)
        out["stage3"] = self.out3(intra)
        return out
