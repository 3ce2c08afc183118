"""C5 FeatureNet backward: how far the GPU's gradients and features are from float64, next to fp32 oracle
runs with image jitter of several sizes (the conditioning of each gradient). One 768x576 view of bench's
C5 inputs, reference-init weights, a seeded normal upstream gradient (as tests/test_gpu_train_c5_featurenet.py).

    python scripts/diag/c5_fnet_grad.py [VIEW] [JITTERS...]     (default 0 2e-7 2e-6 2e-5)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.utils.checkpoint import checkpoint  # noqa: E402

from oracle import transmvs_ref as oracle  # noqa: E402
from transmvsnet_amd import TransMVSNet, synthetic  # noqa: E402
from transmvsnet_amd.featurenet_train import featurenet_train  # noqa: E402

H5, W5, N5 = 576, 768, 4
view = int(sys.argv[1]) if len(sys.argv) > 1 else 0
jits = [float(a) for a in sys.argv[2:]] or [2e-7, 2e-6, 2e-5]
pre = "feature."


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max()) / max(float(np.abs(b).max()), 1e-30)


def dcn_ck(sd, p, x):
    return checkpoint(lambda t: oracle._dcn(sd, p, t), x, use_reentrant=False)


sd0 = synthetic.synthetic_state_dict(synthetic.state_dict_shapes(TransMVSNet()), seed=0, sharpen=100.0)
img = synthetic.synthetic_images(N5, H5, W5, seed=8)[0, view:view + 1]
m = TransMVSNet()
m.load_state_dict(sd0)
m = m.to("cuda").train()
feats = featurenet_train(m.feature, img.cuda())
gu = torch.Generator().manual_seed(100 + view)
dys = [torch.randn(f.shape, generator=gu) for f in feats]
torch.autograd.backward(list(feats), [d.cuda() for d in dys])
torch.cuda.synchronize()
gpu_f = [f.detach().cpu().numpy() for f in feats]
gpu_g = {pre + n: p.grad.detach().cpu().numpy() for n, p in m.feature.named_parameters()}
torch.set_num_threads(min(16, torch.get_num_threads()))


def run(dt, jitter=0.0, seed=1001):
    sd = {k: (v.clone().to(dt) if v.is_floating_point() else v.clone()) for k, v in sd0.items() if k.startswith(pre)}
    for k, v in sd.items():
        if v.is_floating_point() and not k.endswith(("running_mean", "running_var", "num_batches_tracked")):
            v.requires_grad_(True)
    x = img.double()
    if jitter:
        gj = torch.Generator().manual_seed(seed)
        x = x * (1 + jitter * torch.randn(x.shape, generator=gj, dtype=torch.float64))
    out = oracle.feature_net(sd, x.to(dt), training=True, dcn=dcn_ck)
    fs = [out[s] for s in ("stage1", "stage2", "stage3")]
    torch.autograd.backward(fs, [d.to(dt) for d in dys])
    return [f.detach().numpy() for f in fs], {k: v.grad.numpy() for k, v in sd.items() if v.requires_grad}


ex_f, ex_g = run(torch.float64)
print("float64 done", flush=True)
rows = {"gpu": ([rel(a, b) for a, b in zip(gpu_f, ex_f)], {n: rel(gpu_g[n], ex_g[n]) for n in ex_g})}
f, g = run(torch.float32)
rows["fp32"] = ([rel(a, b) for a, b in zip(f, ex_f)], {n: rel(g[n], ex_g[n]) for n in ex_g})
print("fp32 done", flush=True)
for j in jits:
    f, g = run(torch.float32, j)
    rows[f"fp32+{j:g}"] = ([rel(a, b) for a, b in zip(f, ex_f)], {n: rel(g[n], ex_g[n]) for n in ex_g})
    print(f"jitter {j:g} done", flush=True)
print("feature rel. max error vs float64 (stage1, stage2, stage3):")
for k, (fe, _) in rows.items():
    print(f"  {k:14s} " + "  ".join(f"{e:.2e}" for e in fe))
scale = float(np.median([np.abs(v).max() for v in ex_g.values()]))
names = [n for n in sorted(ex_g) if np.abs(ex_g[n]).max() >= 1e-7 * scale]
worst = sorted(names, key=lambda n: -rows["gpu"][1][n])[:12]
print("gradient rel. max error vs float64, worst 12 by the GPU's:")
print("  " + f"{'param':40s}" + "".join(f"{k:>14s}" for k in rows))
for n in worst:
    print("  " + f"{n[8:]:40s}" + "".join(f"{rows[k][1][n]:14.2e}" for k in rows))
print("median over params:", {k: float(np.median([v[1][n] for n in names])) for k, v in rows.items()})
