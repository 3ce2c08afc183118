"""Where the DTU-size depth differences come from: GPU vs the oracle at 16 threads, and the
oracle at 16 threads vs itself at other thread counts (the reference's own run-to-run spread).
Per stage: pixels whose depth differs (>1e-3 mm), mean |d depth|. Usage: l1_origin.py [threads...]"""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
import bench
from oracle import transmvs_ref as oracle
from transmvsnet_amd import TransMVSNet, synthetic

threads = [int(a) for a in sys.argv[1:]] or [16, 1]
H, W, N = bench.H, bench.W, bench.NVIEWS
model = TransMVSNet().eval()
sd = synthetic.synthetic_state_dict(synthetic.state_dict_shapes(model), seed=0, sharpen=100.0)
model.load_state_dict(sd)
feats_cpu, proj, dv = bench.make_inputs(None)
res = {}
if torch.cuda.is_available():
    model = model.cuda()
    with torch.no_grad():
        o = model.forward_features({k: v.cuda() for k, v in feats_cpu.items()}, proj, dv.cuda(), (H, W))
    res["gpu"] = {s: {k: o[s][k].float().cpu() for k in ("depth", "prob_volume")} for s in ("stage1", "stage2", "stage3")}
feats = [{k: v[:, i] for k, v in feats_cpu.items()} for i in range(N)]
for t in threads:
    torch.set_num_threads(t)
    t0 = time.perf_counter()
    with torch.no_grad():
        o = oracle.forward_from_features(sd, feats, proj, dv, (H, W))
    print(f"oracle {t} threads: {time.perf_counter() - t0:.1f} s", flush=True)
    res[f"cpu{t}"] = {s: {k: o[s][k].float() for k in ("depth", "prob_volume")} for s in ("stage1", "stage2", "stage3")}
base = f"cpu{threads[0]}"
for name in res:
    if name == base:
        continue
    for s in ("stage1", "stage2", "stage3"):
        a, b = res[name][s], res[base][s]
        dd = (a["depth"].double() - b["depth"].double()).abs()
        dp = (a["prob_volume"] - b["prob_volume"]).abs().max().item()
        print(f"{name} vs {base} {s}: differing px {int((dd > 1e-3).sum())} / {dd.numel()}  "
              f"mean|dd| {dd.mean().item():.3e}  max|dd| {dd.max().item():.3f}  max|dprob| {dp:.2e}", flush=True)
