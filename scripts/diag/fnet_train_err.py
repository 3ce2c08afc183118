"""The C1 training forward's features (case "i" of tests/golden/train_c1.npz): GPU (featurenet_train,
fmt_train, pathway_train) against the oracle in fp32 (the reference's arithmetic) and fp64 (exact),
per FeatureNet output and per FMT/pathway output, and the stage-3 CostRegNet input (diagnostic, GPU
box)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch

from oracle import transmvs_ref as oracle
from tests._util import golden_rot, golden_state_dict
from tests.test_train_oracle import TRAIN_SHARPEN
from transmvsnet_amd import TransMVSNet, synthetic
from transmvsnet_amd.featurenet_train import featurenet_train
from transmvsnet_amd.train import fmt_train, pathway_train

torch.set_num_threads(16)
H, W, N = 128, 160, 3
sd = golden_state_dict(sharpen=TRAIN_SHARPEN)
m = TransMVSNet(ndepths=[8, 8, 8])
m.load_state_dict(sd)
m = m.cuda().train()
imgs = synthetic.synthetic_images(N, H, W, seed=0)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max())


def report(tag, gpu, r32, r64):
    print(f"{tag:24s} gpu-exact {rel(gpu, r64):.2e}  ref32-exact {rel(r32, r64):.2e}  gpu-ref32 {rel(gpu, r32):.2e}"
          f"  max|exact| {float(r64.abs().max()):.3e}  std {float(r64.double().std()):.3e}", flush=True)


with torch.no_grad(), golden_rot(m):
    sd32 = {k: v.clone() for k, v in sd.items()}
    sd64 = {k: (v.double() if v.is_floating_point() else v.clone()) for k, v in sd.items()}
    f32 = [oracle.feature_net(sd32, imgs[:, v], training=True) for v in range(N)]
    f64 = [oracle.feature_net(sd64, imgs[:, v].double(), training=True) for v in range(N)]
    s1, s2, s3 = featurenet_train(m.feature, imgs[0].cuda())
    for k, g in (("stage1", s1), ("stage2", s2), ("stage3", s3)):
        report(f"FeatureNet {k}", g, torch.cat([f[k] for f in f32]), torch.cat([f[k] for f in f64]))
    p32 = oracle.fmt_with_pathway(sd32, f32)
    p64 = oracle.fmt_with_pathway(sd64, f64)
    st1 = fmt_train(m, s1)
    st2, st3 = pathway_train(m, st1, s2, s3)
    for k, g in (("stage1", st1), ("stage2", st2), ("stage3", st3)):
        report(f"FMT/pathway {k}", g.permute(0, 3, 1, 2), torch.cat([f[k] for f in p32]), torch.cat([f[k] for f in p64]))
