"""Per-layer timing of the inference CostRegNet kernels at the bench's three stage shapes (C2: DTU
864x1152, 48/32/8), each layer launched alone through tmvs_conv3d_mfma (the same kernel instances as
tmvs_costregnet, raw epilogue) and timed with HIP events (median of REPS launches after a warm-up).
Optionally saves / compares every layer's output bit for bit (A/B of library variants: run with
TMVS_LIB_PATH=variants/NAME/libtransmvs_hip.so).

    python scripts/diag/costreg_layers.py [--save out.pt | --compare out.pt] [--reps 20] [--stages 1,2,3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from transmvsnet_amd import ops  # noqa: E402

STAGES = {1: (48, 216, 288), 2: (32, 432, 576), 3: (8, 864, 1152)}
# (name, cin, cout, stride, transposed, input level, skip from)
LAYERS = [("conv0", 1, 8, 1, False, 0, None), ("conv1", 8, 16, 2, False, 0, None), ("conv2", 16, 16, 1, False, 1, None),
          ("conv3", 16, 32, 2, False, 1, None), ("conv4", 32, 32, 1, False, 2, None), ("conv5", 32, 64, 2, False, 2, None),
          ("conv6", 64, 64, 1, False, 3, None), ("conv7", 64, 32, 2, True, 3, "conv4"),
          ("conv9", 32, 16, 2, True, 2, "conv2"), ("conv11", 16, 8, 2, True, 1, "conv0"), ("prob", 8, 1, 1, False, 0, None)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--compare")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--stages", default="1,2,3")
    ap.add_argument("--layers", default="")
    a = ap.parse_args()
    dev = torch.device("cpu") if os.environ.get("TMVS_DRYRUN") else torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    outs, total = {}, 0.0
    ref = torch.load(a.compare, weights_only=True) if a.compare else None
    only = set(a.layers.split(",")) if a.layers else None
    for s in map(int, a.stages.split(",")):
        d, h, w = STAGES[s]
        acts = {}
        line = []
        for name, ci, co, st, tr, lvl, skip in LAYERS:
            dd, hh, ww = d >> lvl, h >> lvl, w >> lvl
            x = torch.randn(1, dd, hh, ww, ci, generator=g).clamp_min(0).to(dev)
            wt = (torch.randn(27, co, ci, generator=g) * (1.0 / (27 * ci) ** 0.5)).to(dev)
            if (ci, co) == (8, 1):  # prob's packing (ops.prob_pack): [3 kh][72]
                wt = wt.reshape(3, 72).contiguous()
            sk = None
            if skip:
                lv = {"conv4": 2, "conv2": 1, "conv0": 0}[skip]
                sk = torch.randn(1, d >> lv, h >> lv, w >> lv, co, generator=g).to(dev)
            acts[name] = (x, wt, sk)
        torch.cuda.synchronize()
        for name, ci, co, st, tr, lvl, skip in LAYERS:
            if only and name not in only:
                continue
            x, wt, sk = acts[name]
            y = ops.conv3d_mfma(x, wt, co, st, transposed=tr, skip=sk)  # warm-up
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                y = ops.conv3d_mfma(x, wt, co, st, transposed=tr, skip=sk)
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
            us = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ts)[len(ts) // 2]
            total += us
            key = f"s{s}_{name}"
            outs[key] = y.cpu()
            same = ""
            if ref is not None and key in ref:
                same = " ==" if torch.equal(ref[key], outs[key]) else f" DIFF {float((ref[key] - outs[key]).abs().max()):.2e}"
            line.append(f"{name} {us:7.1f}{same}")
        print(f"stage {s}: " + " | ".join(line), flush=True)
    print(f"total {total:.1f} us over the listed layers")
    if a.save:
        torch.save(outs, a.save)


if __name__ == "__main__":
    main()
