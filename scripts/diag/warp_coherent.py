"""The stage-2/3 cost-volume launches on coherent hypotheses next to the bench's own (bench.coherent_warp_timing,
the secondary roofline_kernels entry of the bench line), standalone.

    python scripts/diag/warp_coherent.py [REPS] [--json OUT]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from transmvsnet_amd import TransMVSNet, synthetic  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else 20
dev = torch.device("cuda", 0)
m = TransMVSNet().eval()
m.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=0, sharpen=100.0))
m = m.to(dev)
feats_cpu, proj, dv = bench.make_inputs(dev)
res = bench.coherent_warp_timing(m, {k: v.to(dev) for k, v in feats_cpu.items()}, proj, dv.to(dev), reps)
print(json.dumps(res, indent=1))
if "--json" in sys.argv:
    out = sys.argv[sys.argv.index("--json") + 1]
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
