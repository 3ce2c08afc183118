"""Stage-1 argmax flips between the GPU and the fp32 oracle at a full-size shape, and which side of
the tie exact arithmetic is on (diagnostic, GPU box). Default: C4's shape, TnT 1056x1920, N=11
(test_gpu_fullsize.py's inputs: stacked_features seed 2, synthetic_cameras seed 1).

For every stage-1 pixel whose WTA depth differs between the GPU forward and the fp32 oracle:
  * the reference's own fp32 spread: the oracle's cost volume + CostRegNet at 1, 4 and 16 torch
    threads (MKL/oneDNN blocking changes with the thread count) -> argmax and log-prob margin;
  * component swaps: the GPU's FMT features, or the GPU's cost volume, inside the oracle stage;
  * exact arithmetic: FMT, cost volume (incl. PixelwiseNet) and CostRegNet in float64 from the same
    fp32 inputs and weights -> argmax and margin.
Writes a JSON summary (argv[1], default gpurun_out/stage1_flip.json) beside the log lines.
"""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch

from oracle import transmvs_ref as oracle
from transmvsnet_amd import TransMVSNet, synthetic

NT = int(os.environ.get("THREADS", "16"))
torch.set_num_threads(NT)
N = int(os.environ.get("NVIEWS", "11"))
H, W = int(os.environ.get("H", "1056")), int(os.environ.get("W", "1920"))
OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stage1_flip.json"


def log(*a):
    print(*a, flush=True)


def top2(col):
    """(argmax, log-prob margin top1 - top2) of one pixel's logits [D] in float64."""
    x = col.double()
    lp = x - torch.logsumexp(x, 0)
    s = torch.sort(lp, descending=True).values
    return int(torch.argmax(col)), float(s[0] - s[1])


model = TransMVSNet().eval()
sd = synthetic.synthetic_state_dict(synthetic.state_dict_shapes(model), seed=0, sharpen=100.0)
sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
model.load_state_dict(sd)
model = model.cuda()
feats_cpu = synthetic.stacked_features(N, H, W, seed=2)
proj = synthetic.synthetic_cameras(N, H, W, seed=1)
dv = synthetic.synthetic_depth_values(1)
feats = [{k: v[:, i] for k, v in feats_cpu.items()} for i in range(N)]
P = "cost_regularization.0."

with torch.no_grad():
    out = model.forward_features({k: v.cuda() for k, v in feats_cpu.items()}, proj, dv.cuda(), (H, W))
    torch.cuda.synchronize()
    g_depth = out["stage1"]["depth"].cpu()
    g_prob = out["stage1"]["prob_volume"].cpu()
    log("GPU forward done")
    f32 = oracle.fmt_with_pathway(sd, feats)
    hyp = oracle.stage_hypotheses(None, dv, 0, (H, W))
    fs = [f["stage1"] for f in f32]
    sim32, _ = oracle.build_cost_volume(sd, fs, proj["stage1"], hyp)
    lg32 = oracle.cost_reg_net(sd, P, sim32)
    prob32, dep32, _ = oracle.softmax_regression(lg32, hyp)
    log("oracle stage 1 done")
    diff = (g_depth.double() - dep32.clamp(*oracle.DEPTH_CLAMP).double()).abs().numpy() > 1e-3
    px = [tuple(int(t) for t in f) for f in np.argwhere(diff)]
    log(f"stage-1 pixels differing: {len(px)} {px}")
    report = {"shape": [N, H, W], "threads": NT, "pixels": []}
    if px:
        # GPU FMT features into the oracle stage (swap), GPU-identical cost volume from a GPU run of
        # stage 1 alone is not exposed, so the feature swap isolates FMT vs (cost volume + CostRegNet)
        st1 = model._fmt(feats_cpu["stage1"][0].cuda(), model._prepared(torch.device("cuda", 0)))
        h1, w1 = H // 4, W // 4
        gf = [st1.view(N, h1, w1, 32)[i:i + 1].permute(0, 3, 1, 2).cpu() for i in range(N)]
        sim_f, _ = oracle.build_cost_volume(sd, gf, proj["stage1"], hyp)
        lg_f = oracle.cost_reg_net(sd, P, sim_f)
        log("feature swap done")
        spread = {}
        for nt in (1, 4):
            torch.set_num_threads(nt)
            sim_t, _ = oracle.build_cost_volume(sd, fs, proj["stage1"], hyp)
            spread[nt] = oracle.cost_reg_net(sd, P, sim_t)
            log(f"oracle at {nt} threads done")
        torch.set_num_threads(NT)
        f64 = oracle.fmt_with_pathway(sd64, [{k: v.double() for k, v in f.items()} for f in feats])
        log("fp64 features done")
        p64 = {k: v.double() for k, v in proj.items()}
        sim64, _ = oracle.build_cost_volume(sd64, [f["stage1"] for f in f64], p64["stage1"], hyp.double())
        lg64 = oracle.cost_reg_net(sd64, P, sim64)
        lg64c = oracle.cost_reg_net(sd64, P, sim32.double())
        log("fp64 stage 1 done")
        for (b, y, x) in px:
            col = lambda t: t[b, 0, :, y, x] if t.dim() == 5 else t[b, :, y, x]
            gp = g_prob[b, :, y, x].double()
            gs = torch.sort(torch.log(gp.clamp_min(1e-30)), descending=True).values
            ent = {"y": y, "x": x, "ref32_depth": float(dep32[b, y, x]), "gpu_depth": float(g_depth[b, y, x]),
                   "gpu_argmax": int(torch.argmax(gp)), "gpu_margin": float(gs[0] - gs[1])}
            log(f"pixel (y={y}, x={x}): ref32 depth {ent['ref32_depth']:.4f}  gpu depth {ent['gpu_depth']:.4f}  "
                f"GPU argmax {ent['gpu_argmax']} margin {ent['gpu_margin']:.3e}")
            for tag, t in (("ref32_%dthr" % NT, lg32), ("ref32_1thr", spread[1]), ("ref32_4thr", spread[4]),
                           ("swap_gpu_features", lg_f), ("fp64_whole_stage", lg64), ("fp64_costreg_of_ref32_sim", lg64c)):
                a, m = top2(col(t))
                srt = torch.sort(col(t).double(), descending=True)
                ent[tag] = {"argmax": a, "margin": m, "top2": [int(i) for i in srt.indices[:2]],
                            "top2_logits": [float(v) for v in srt.values[:2]]}
                log(f"  {tag:28s}: argmax {a}  margin {m:.3e}  top2 {ent[tag]['top2']} {ent[tag]['top2_logits']}")
            report["pixels"].append(ent)
    os.makedirs(os.path.dirname(OUT) or ".", exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(report, f, indent=1)
    log("wrote", OUT)
