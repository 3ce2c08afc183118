"""Conditioning of the C1 training step's gradients (case "i" of tests/golden/train_c1.npz): the
oracle in fp32 at different torch thread counts (different MKL/oneDNN blocking = different fp32
rounding of the SAME arithmetic) against fp64, for the gradients the GPU test flags. If two fp32
evaluations of the reference's own arithmetic disagree with fp64 by the GPU's margin, the gradient is
ill-conditioned rather than mis-computed (diagnostic; CPU only)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch

from tests.test_train_oracle import GOLD, train_step_oracle

NAMES = ["cost_regularization.2.conv5.bn.bias", "cost_regularization.2.conv5.conv.weight",
         "cost_regularization.2.conv4.conv.weight", "FMT_with_pathway.FMT.layers.7.linear2.weight",
         "FMT_with_pathway.FMT.layers.7.attention.query_projection.bias", "feature.out2.5.weight"]
g = {k: v for k, v in np.load(GOLD).items()}
case = sys.argv[1] if len(sys.argv) > 1 else "i"
ex = train_step_oracle(g, case, dtype=torch.float64)[2]
rows = {n: [] for n in NAMES}
for nt in (1, 2, 4, 16):
    torch.set_num_threads(nt)
    sd = train_step_oracle(g, case)[2]
    for n in NAMES:
        a = sd[n].grad.double().numpy()
        b = ex[n].grad.double().numpy()
        rows[n].append((nt, float(np.abs(a - b).max() / np.abs(b).max())))
for n in NAMES:
    f = g[f"{case}_grad.{n}"].astype(np.float64)
    b = ex[n].grad.double().numpy()
    print(f"{n:62s} fixture {float(np.abs(f - b).max() / np.abs(b).max()):.1e}  "
          + "  ".join(f"{nt}thr {e:.1e}" for nt, e in rows[n]), flush=True)
# ~1-ulp input jitter (train_step_oracle's perturb_seed): the fp32 spread the GPU test's bar uses
torch.set_num_threads(16)
for seed in range(6):
    sd = train_step_oracle(g, case, perturb_seed=1000 + seed)[2]
    print(f"jitter seed {seed}: " + "  ".join(
        f"{n.split('.', 1)[-1][-28:]} {float(np.abs(sd[n].grad.double().numpy() - ex[n].grad.double().numpy()).max() / np.abs(ex[n].grad.double().numpy()).max()):.1e}"
        for n in NAMES), flush=True)
