"""Bitwise A/B of the hot path's outputs between two builds of the library (run once per build).

    TMVS_LIB_PATH=variants/X/libtransmvs_hip.so python scripts/diag/out_bits.py OUT.npz
    python scripts/diag/out_bits.py --compare A.npz B.npz

Dumps the FMT tokens and every stage's depth / confidence / prob volume of one synthetic C2 depth
map (bench.py's inputs and weights); --compare reports the max |difference| and the count of
differing elements per array (0 everywhere = the two builds are bit-identical on this input).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    worst = 0
    for k in a.files:
        d = np.abs(a[k].astype(np.float64) - b[k].astype(np.float64))
        n = int((a[k] != b[k]).sum())
        worst = max(worst, n)
        print(f"{k:24s} differing {n:10d} of {a[k].size:10d}  max|d| {d.max():.3e}")
    print("BITWISE IDENTICAL" if worst == 0 else "DIFFERENT")
    sys.exit(0)

import torch  # noqa: E402

import bench  # noqa: E402
from transmvsnet_amd import TransMVSNet, synthetic  # noqa: E402

dev = torch.device("cuda:0")
model = TransMVSNet().eval()
model.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(model), seed=0, sharpen=100.0))
model = model.to(dev)
feats_cpu, proj, dv = bench.make_inputs(dev)
feats = {k: v.to(dev) for k, v in feats_cpu.items()}
with torch.no_grad():
    out = model.forward_features(feats, proj, dv.to(dev), (bench.H, bench.W))
    tokens = model._fmt(feats["stage1"][0], model._prepared(dev))
torch.cuda.synchronize()
arrs = {"fmt_tokens": tokens.cpu().numpy()}
for s in ("stage1", "stage2", "stage3"):
    for k in ("depth", "photo_confidence", "prob_volume"):
        arrs[f"{s}_{k}"] = out[s][k].cpu().numpy()
np.savez(sys.argv[1], **arrs)
print("wrote", sys.argv[1])
