"""Weight re-layouts of a training step as ONE gather.

The HIP kernels read weights in their own layouts ([27][Co][Ci] taps, flipped taps for a data gradient,
prob_kernel's [3][72], the FMT's transposed linears, ...), and the weight gradients come back in the
kernels' layouts too. Each re-layout is a pure permutation (with zero padding) of a parameter, so
instead of one permute/flip/cat launch per tensor (100+ small launches in a C5 step) the permutation
is evaluated once on an index tensor -- fn(arange) gives, per packed element, the flat index of its
source -- and every later call is cat(params) + one index gather. Index 0 is a zero slot (padding).
"""
from __future__ import annotations

import math

import torch

_IDX = {}


def gather_packs(tensors, specs, key):
    """tensors: list of tensors; specs: list of (i, fn), fn a permutation / reshape / flip / zero-padding
    / concatenation of tensors[i] (i an int, or a tuple of ints: fn(*those tensors)) -- no arithmetic;
    key: a hashable naming the specs (the tensors' shapes are added to it).
    -> [fn(tensors[i]) for (i, fn) in specs], computed with one cat and one index gather."""
    dev = tensors[0].device
    full_key = (key, tuple(tuple(t.shape) for t in tensors), str(dev))
    ent = _IDX.get(full_key)
    if ent is None:
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            # inside a capture the index kernels would only be recorded, and the uninitialised index
            # tensor cached for every later eager call
            raise RuntimeError(f"gather_packs: index for {key!r} not built yet inside a HIP-graph capture; "
                               "run the step once eagerly before capturing it")
        offs, off = [], 1
        for t in tensors:
            offs.append(off)
            off += t.numel()
        if off >= (1 << 24):
            raise ValueError("gather_packs: more elements than fp32 indices hold exactly")
        idxs, shapes = [], []
        with torch.no_grad():
            ars = [torch.arange(o, o + t.numel(), device=dev, dtype=torch.float32).view(t.shape)
                   for o, t in zip(offs, tensors)]
            for i, fn in specs:
                packed = fn(*[ars[j] for j in i]) if isinstance(i, tuple) else fn(ars[i])
                idxs.append(packed.reshape(-1).round().long())
                shapes.append(tuple(packed.shape))
        ent = (torch.cat(idxs), shapes)
        _IDX[full_key] = ent
    idx, shapes = ent
    with torch.no_grad():
        src = torch.cat([tensors[0].new_zeros(1, dtype=torch.float32)] +
                        [t.detach().float().reshape(-1) for t in tensors])
        flat = src[idx]
    outs, o = [], 0
    for s in shapes:
        n = math.prod(s)
        outs.append(flat[o:o + n].view(s))
        o += n
    return outs
