"""Drive tmvs_costregnet_wta at the DTU stage-2 / stage-3 shapes (C2: 32x432x576, 8x864x1152) REPS times --
the program the fused conv11 + prob kernel's PMC passes and traces run over (scripts/pmc_kernel.sh PMC_PROG).

    python scripts/diag/dp_run.py [REPS]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from transmvsnet_amd import TransMVSNet, ops, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
m = TransMVSNet().eval()
m.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=0, sharpen=100.0))
m = m.cuda()
g = torch.Generator().manual_seed(0)
for s, (d, h, w) in ((1, (32, 432, 576)), (2, (8, 864, 1152))):
    st, _keep = m.cost_regularization[s].packed(torch.device("cuda"))
    x = torch.randn(1, d, h, w, generator=g).cuda()
    hyp = (425.0 + torch.rand(1, d, h, w, generator=g).mul(510.0)).sort(dim=1).values.cuda()
    for _ in range(reps):
        ops.costregnet_wta(x, st, hyp, (425.0, 935.0))
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        ops.costregnet_wta(x, st, hyp, (425.0, 935.0))
    ev[1].record()
    torch.cuda.synchronize()
    print(f"stage {s + 1} {d}x{h}x{w}: costregnet_wta {ev[0].elapsed_time(ev[1]) / reps * 1e3:.1f} us", flush=True)
