"""C4 shape (TnT 1056x1920, N=11), stage 1 in fp32 and in float64 through the oracle (CPU only; runs in
the build container): the near-tie pixels of the fp32 reference (top-2 log-prob margin < 1e-3) with the
fp32 and the exact (fp64: FMT, cost volume incl. PixelwiseNet, CostRegNet from the same fp32 inputs and
weights) argmax and margins. A GPU stage-1 flip at one of these pixels is then attributed by lookup:
if fp64 picks the GPU's index, the fp32 reference's pick is the rounding artefact.

    python scripts/diag/c4_stage1_exact.py OUT.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from oracle import transmvs_ref as oracle
from transmvsnet_amd import TransMVSNet, synthetic

N, H, W = 11, 1056, 1920
torch.set_num_threads(int(os.environ.get("THREADS", str(os.cpu_count() or 8))))
out_path = sys.argv[1] if len(sys.argv) > 1 else "c4_stage1_exact.json"
sd = synthetic.synthetic_state_dict(synthetic.state_dict_shapes(TransMVSNet()), seed=0, sharpen=100.0)
feats_cpu = synthetic.stacked_features(N, H, W, seed=2)
proj = synthetic.synthetic_cameras(N, H, W, seed=1)
dv = synthetic.synthetic_depth_values(1)
P = "cost_regularization.0."


def log(*a):
    print(*a, flush=True)


def stage1_logits(sd_, feats, proj_, dv_):
    # FMT_with_pathway's stage-1 output (models/FMT.py:212-226): the FMT part of oracle.fmt_with_pathway
    pre = "FMT_with_pathway.FMT."
    ref_list = oracle.fmt_ref(sd_, feats[0]["stage1"].clone(), pre)
    f = [ref_list[-1]] + [oracle.fmt_src(sd_, [r.clone() for r in ref_list], x["stage1"].clone(), pre) for x in feats[1:]]
    log("  features done")
    hyp = oracle.stage_hypotheses(None, dv_, 0, (H, W))
    sim, _ = oracle.build_cost_volume(sd_, f, proj_["stage1"], hyp)
    log("  cost volume done")
    return oracle.cost_reg_net(sd_, P, sim)[:, 0], hyp


def margins(lg):
    x = lg.double()
    lp = x - torch.logsumexp(x, 1, keepdim=True)
    top = torch.topk(lp, 2, dim=1)
    return top.indices, (top.values[:, 0] - top.values[:, 1])


with torch.no_grad():
    feats = [{"stage1": feats_cpu["stage1"][:, i]} for i in range(N)]
    log("fp32 stage 1")
    lg32, hyp = stage1_logits(sd, feats, proj, dv)
    idx32, m32 = margins(lg32)
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    log("fp64 stage 1")
    lg64, _ = stage1_logits(sd64, [{"stage1": f["stage1"].double()} for f in feats],
                           {k: v.double() for k, v in proj.items()}, dv.double())
    idx64, m64 = margins(lg64)
    near = torch.nonzero(m32[0] < 1e-3)
    rows = []
    for y, x in near.tolist():
        rows.append({"y": y, "x": x, "fp32_top2": idx32[0, :, y, x].tolist(), "fp32_margin": float(m32[0, y, x]),
                     "fp64_top2": idx64[0, :, y, x].tolist(), "fp64_margin": float(m64[0, y, x]),
                     "fp32_depth": float(hyp[0, idx32[0, 0, y, x], y, x]), "fp64_depth": float(hyp[0, idx64[0, 0, y, x], y, x])})
    disagree = int((idx32[0, 0] != idx64[0, 0]).sum())
    res = {"shape": [N, H, W], "threads": torch.get_num_threads(),
           "pixels_fp32_vs_fp64_argmax_differ": disagree, "near_ties_fp32_margin_lt_1e-3": rows}
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    log(f"{len(rows)} near ties; fp32 vs fp64 argmax differ at {disagree} pixels; wrote {out_path}")
