"""Training path, first differentiable block: CostRegNet in train
mode with its backward on the HIP kernels of csrc/costreg_train.hip.

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

# (name, stride, transposed, skip source) in forward order; channels from the module
_LAYERS = (("conv0", 1, False, None), ("conv1", 2, False, None), ("conv2", 1, False, None),
           ("conv3", 2, False, None), ("conv4", 1, False, None), ("conv5", 2, False, None),
           ("conv6", 1, False, None), ("conv7", 2, True, "conv4"), ("conv9", 2, True, "conv2"),
           ("conv11", 2, True, "conv0"))
BN_MOMENTUM = 0.1


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
        acts = {"input": (x.contiguous().view(b, d, h, w, 1), (d, h, w))}
        saved = []
        cur, dims = acts["input"]
        stats = []
        for i, (name, stride, transposed, skip) in enumerate(_LAYERS):
            wt, g, bt = ws[3 * i], ws[3 * i + 1], ws[3 * i + 2]
            cout = wt.shape[1] if transposed else wt.shape[0]
            odims = tuple(2 * n for n in dims) if transposed else (dims if stride == 1 else _down(dims))
            z = ops.conv3d_generic(cur, _pack_fwd(wt.detach(), transposed), cout, odims, stride, transposed)
            mean, var = ops.bn_stats(z)
            y = ops.bn_relu_train(z, mean, var, g.detach(), bt.detach(), eps,
                                  skip=acts[skip][0] if skip is not None else None)
            saved.append((cur, dims, z, mean, var))
            stats.append((mean, var, z.numel() // z.shape[-1]))
            acts[name] = (y, odims)
            cur, dims = y, odims
        logits = ops.conv3d_generic(cur, _pack_fwd(wprob.detach(), False), 1, dims, 1, False)
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
        grads[-1] = _unpack_wgrad(ops.conv3d_wgrad(g, ctx.u11, 1), wprob.shape)
        # gradient w.r.t. each layer's output, filled as the backward reaches it
        dout = {"conv11": ops.conv3d_generic(g, _pack_dgrad(wprob.detach(), False), ctx.u11.shape[-1], (d, h, w), 1,
                                             transposed=True)}
        for i in range(len(_LAYERS) - 1, -1, -1):
            name, stride, transposed, skip = _LAYERS[i]
            wt, gm, bt = ws[3 * i], ws[3 * i + 1], ws[3 * i + 2]
            xin, idims, z, mean, var = ctx.layer_io[i]
            dy = dout.pop(name)
            if skip is not None:  # y = skip + relu(bn(z)): the skip source receives dy as is
                dout[skip] = dy.clone() if skip not in dout else dout[skip].add_(dy)
            dz, dgam, dbet = ops.bn_relu_backward(dy, z, mean, var, gm.detach(), bt.detach(), eps)
            if transposed:
                dw = ops.conv3d_wgrad(xin, dz, 2)
            else:
                dw = ops.conv3d_wgrad(dz, xin, stride)
            grads[3 * i] = _unpack_wgrad(dw, wt.shape)
            grads[3 * i + 1], grads[3 * i + 2] = dgam, dbet
            prev = _LAYERS[i - 1][0] if i > 0 else "input"
            cin = xin.shape[-1]
            acc = dout.get(prev)
            if transposed:   # dgrad of ConvTranspose3d: strided gather of dz
                dx = ops.conv3d_generic(dz, _pack_dgrad(wt.detach(), True), cin, idims, 2, False, out=acc)
            else:            # dgrad of Conv3d: transposed gather of dz
                dx = ops.conv3d_generic(dz, _pack_dgrad(wt.detach(), False), cin, idims, stride, True, out=acc)
            dout[prev] = dx
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
        with torch.no_grad():
            for (name, _, _, _), (mean, var, n) in zip(_LAYERS, stats):
                bn = getattr(module, name).bn
                bn.running_mean.mul_(1.0 - BN_MOMENTUM).add_(mean, alpha=BN_MOMENTUM)
                bn.running_var.mul_(1.0 - BN_MOMENTUM).add_(var * (n / max(n - 1, 1)), alpha=BN_MOMENTUM)
                bn.num_batches_tracked.add_(1)
    return logits
