"""Where do the GPU-vs-reference depth flips at DTU size come from? (diagnostic, GPU box)

For stages 2 and 3 (each from the oracle's previous-stage depth, so no cascade), swap ONE component
of the oracle's stage computation for the GPU's and count the depth pixels that then differ from the
pure oracle, with the reference top-2 log-prob margin of each differing pixel:
  feat : GPU FMT+pathway features -> oracle warp/corr + CostRegNet + softmax
  warp : oracle features -> GPU warp/corr (fused cost volume) -> oracle CostRegNet + softmax
  creg : oracle similarity volume -> GPU CostRegNet -> oracle softmax
  all  : the GPU stage (tmvs_depth_stage) on the GPU features
"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch
import torch.nn.functional as F

import bench
from oracle import transmvs_ref as oracle
from transmvsnet_amd import TransMVSNet, ops, synthetic
from transmvsnet_amd.model import DEPTH_CLAMP, STAGE_SCALES

torch.set_num_threads(16)
H, W, N = bench.H, bench.W, int(os.environ.get("NVIEWS", bench.NVIEWS))
model = TransMVSNet().eval()
sd = synthetic.synthetic_state_dict(synthetic.state_dict_shapes(model), seed=0, sharpen=100.0)
model.load_state_dict(sd)
model = model.cuda()
feats_cpu = synthetic.stacked_features(N, H, W, seed=2)
proj = synthetic.synthetic_cameras(N, H, W, seed=1)
dv = synthetic.synthetic_depth_values(1)
feats = [{k: v[:, i] for k, v in feats_cpu.items()} for i in range(N)]


def margins(prob):
    srt = np.sort(prob.numpy().astype(np.float64), axis=1)
    return np.log(np.maximum(srt[:, -1], 1e-30)) - np.log(np.maximum(srt[:, -2], 1e-30))


def report(tag, depth, ref_depth, marg):
    d = np.abs(depth.cpu().numpy().astype(np.float64) - ref_depth.numpy().astype(np.float64))
    diff = d > 1e-3
    m = np.sort(marg[diff])
    print(f"  {tag:5s}: differing {int(diff.sum()):4d}  mean|dd| {d.mean():.3e}  margins of flips "
          f"{np.array2string(m[:12], precision=5)}{' ...' if m.size > 12 else ''}  max {m.max() if m.size else 0:.2e}",
          flush=True)


with torch.no_grad():
    prep = model._prepared(torch.device("cuda"))
    f32 = oracle.fmt_with_pathway(sd, feats)
    s1 = feats_cpu["stage1"][0].cuda()
    st1 = model._fmt(s1, prep).view(N, H // 4, W // 4, 32)
    st2 = ops.fmt_pathway(st1, feats_cpu["stage2"][0].cuda(), prep["red1"], prep["sm1"])
    st3 = ops.fmt_pathway(st2, feats_cpu["stage3"][0].cuda(), prep["red2"], prep["sm2"])
    gpu_feat = (st1, st2, st3)
    depth = None
    vw = None
    for s in range(3):
        name = f"stage{s + 1}"
        hyp = oracle.stage_hypotheses(depth, dv, s, (H, W))
        vw_up = vw
        if s > 0:
            for _ in range(s):
                vw_up = F.interpolate(vw_up, scale_factor=2, mode="nearest")
        fs = [f[name] for f in f32]
        sim, vw_new = oracle.build_cost_volume(sd, fs, proj[name], hyp, vw_up)
        lg = oracle.cost_reg_net(sd, f"cost_regularization.{s}.", sim)
        prob, dep, conf = oracle.softmax_regression(lg, hyp)
        marg = margins(prob)
        ref_depth = dep.clamp(*DEPTH_CLAMP)
        print(f"{name}: max|logit| {lg.abs().max().item():.1f}  pixels with margin < 1e-4: {(marg < 1e-4).sum()}  "
              f"< 1e-3: {(marg < 1e-3).sum()}", flush=True)
        if s > 0:
            rows = ops.proj_rows(proj[name])
            # feat: GPU features through the oracle
            gf = [gpu_feat[s][i:i + 1].permute(0, 3, 1, 2).cpu() for i in range(N)]
            sim_f, _ = oracle.build_cost_volume(sd, gf, proj[name], hyp, vw_up)
            p_f, d_f, _ = oracle.softmax_regression(oracle.cost_reg_net(sd, f"cost_regularization.{s}.", sim_f), hyp)
            report("feat", d_f.clamp(*DEPTH_CLAMP), ref_depth, marg)
            # warp: oracle features through the GPU cost volume
            fs_g = torch.cat(fs, 0).permute(0, 2, 3, 1).contiguous().cuda()
            sim_g, _, _ = ops.warp_corr(fs_g[0:1], fs_g[1:].unsqueeze(0), rows[0:1], hyp.cuda().contiguous(),
                                        view_w_in=vw.cuda().contiguous(), vw_shift=s)
            print(f"  warp sim: max|gpu-ref| {(sim_g.cpu() - sim[:, 0]).abs().max().item():.2e}  "
                  f"bit-exact {(sim_g.cpu() == sim[:, 0]).float().mean().item():.4f}", flush=True)
            p_w, d_w, _ = oracle.softmax_regression(
                oracle.cost_reg_net(sd, f"cost_regularization.{s}.", sim_g.cpu().unsqueeze(1)), hyp)
            report("warp", d_w.clamp(*DEPTH_CLAMP), ref_depth, marg)
            # creg: oracle similarity through the GPU CostRegNet
            lg_g = ops.costregnet(sim[:, 0].contiguous().cuda(), prep["cr"][s][0])
            print(f"  logits: max|gpu-ref| {(lg_g.cpu() - lg[:, 0]).abs().max().item():.2e}", flush=True)
            p_c, d_c, _ = oracle.softmax_regression(lg_g.cpu().unsqueeze(1), hyp)
            report("creg", d_c.clamp(*DEPTH_CLAMP), ref_depth, marg)
            # all: the GPU stage on GPU features from the oracle's previous depth
            prev = torch.gather(prev_hyp, 1, prev_prob.argmax(1, keepdim=True)).squeeze(1)
            o, _ = ops.depth_stage(dv.cuda(), prev.cuda().contiguous(), gpu_feat[s], model.ndepths[s],
                                   model.depth_interals_ratio[s], (H, W), STAGE_SCALES[s], rows[0], None,
                                   vw.cuda().contiguous(), s, prep["cr"][s][0], DEPTH_CLAMP)
            report("all", o["depth"].cpu(), ref_depth, marg)
        if s == 0:
            vw = vw_new
        depth = dep
        prev_hyp, prev_prob = hyp, prob
