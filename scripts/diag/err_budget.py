"""Error budget of the GPU path against the oracle at DTU size, one component at a time, each fed
the oracle's own inputs: FMT+pathway features, stage-1 similarity, stage-1 CostRegNet logits.
Each is also compared with a float64 evaluation of the oracle (the exact value)."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
import bench
from oracle import transmvs_ref as oracle
from transmvsnet_amd import TransMVSNet, ops, synthetic

torch.set_num_threads(16)
H, W, N = bench.H, bench.W, bench.NVIEWS
if os.environ.get("SMALL"):
    H, W = bench.H, bench.W = 128, 160
model = TransMVSNet().eval()
sd = synthetic.synthetic_state_dict(synthetic.state_dict_shapes(model), seed=0, sharpen=100.0)
model.load_state_dict(sd)
model = model.cuda()
sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
feats_cpu, proj, dv = bench.make_inputs(None)
feats = [{k: v[:, i] for k, v in feats_cpu.items()} for i in range(N)]


def md(a, b):
    return (a.double().cpu() - b.double().cpu()).abs().max().item()


with torch.no_grad():
    prep = model._prepared(torch.device("cuda"))
    f32 = oracle.fmt_with_pathway(sd, feats)
    f64 = oracle.fmt_with_pathway(sd64, [{k: v.double() for k, v in f.items()} for f in feats])
    s1 = feats_cpu["stage1"][0].cuda()
    tok = model._fmt(s1, prep)
    h1, w1 = H // 4, W // 4
    st1 = tok.view(N, h1, w1, 32)
    st2 = ops.fmt_pathway(st1, feats_cpu["stage2"][0].cuda(), prep["red1"], prep["sm1"])
    st3 = ops.fmt_pathway(st2, feats_cpu["stage3"][0].cuda(), prep["red2"], prep["sm2"])
    for name, g in (("stage1", st1), ("stage2", st2), ("stage3", st3)):
        o32 = torch.stack([f[name] for f in f32]).squeeze(1).permute(0, 2, 3, 1)
        o64 = torch.stack([f[name] for f in f64]).squeeze(1).permute(0, 2, 3, 1)
        print(f"features {name}: |gpu-ref32| {md(g, o32):.2e}  |gpu-exact| {md(g, o64):.2e}  |ref32-exact| {md(o32, o64):.2e}",
              flush=True)
    # stage 1 cost volume from the oracle's features
    hyp = oracle.stage_hypotheses(None, dv, 0, (H, W))
    fs = [f["stage1"] for f in f32]
    sim32, vw32 = oracle.build_cost_volume(sd, fs, proj["stage1"], hyp)
    sim64, _ = oracle.build_cost_volume(sd64, [f.double() for f in fs], proj["stage1"].double(), hyp.double())
    fs_g = torch.stack(fs).squeeze(1).permute(0, 2, 3, 1).contiguous().cuda()
    rows = ops.proj_rows(proj["stage1"])
    hyp_g = hyp.cuda().contiguous()
    sim_g, _, vw_g = ops.warp_corr(fs_g[0:1], fs_g[1:].unsqueeze(0), rows[0:1], hyp_g, pw_params=prep["pw"])
    print(f"stage1 sim: |gpu-ref32| {md(sim_g, sim32[:, 0]):.2e}  |gpu-exact| {md(sim_g, sim64[:, 0]):.2e}  "
          f"|ref32-exact| {md(sim32, sim64):.2e}  max|sim| {sim32.abs().max().item():.2f}", flush=True)
    lg32 = oracle.cost_reg_net(sd, "cost_regularization.0.", sim32)
    lg64 = oracle.cost_reg_net(sd64, "cost_regularization.0.", sim32.double())
    lg_g = ops.costregnet(sim32[:, 0].contiguous().cuda(), prep["cr"][0][0])
    print(f"stage1 logits (same sim): |gpu-ref32| {md(lg_g, lg32[:, 0]):.2e}  |gpu-exact| {md(lg_g, lg64[:, 0]):.2e}  "
          f"|ref32-exact| {md(lg32, lg64):.2e}  max|logit| {lg32.abs().max().item():.1f}", flush=True)
    # whole forward: GPU and the fp32 oracle, each against the float64 oracle (the exact answer)
    out_g = model.forward_features({k: v.cuda() for k, v in feats_cpu.items()}, proj, dv.cuda(), (H, W))
    ref32 = oracle.forward_from_features(sd, feats, proj, dv, (H, W))
    ex = oracle.forward_from_features(sd64, [{k: v.double() for k, v in f.items()} for f in feats],
                                      {k: v.double() for k, v in proj.items()}, dv.double(), (H, W))
    for s in ("stage1", "stage2", "stage3"):
        e = ex[s]["depth"].double()
        for nm, o in (("gpu", out_g[s]["depth"].cpu()), ("ref32", ref32[s]["depth"])):
            dd = (o.double() - e).abs()
            print(f"{s} {nm} vs exact: differing px {int((dd > 1e-3).sum())}  mean|dd| {dd.mean().item():.3e}", flush=True)
        dd = (out_g[s]["depth"].cpu().double() - ref32[s]["depth"].double()).abs()
        print(f"{s} gpu vs ref32: differing px {int((dd > 1e-3).sum())}  mean|dd| {dd.mean().item():.3e}", flush=True)
