"""Tanks&Temples-size forward (config C4 shape, 1056x1920, N=11) on one GPU: FeatureNet + hot path
from images. Checks the outputs are finite and in range, times the full forward (HIP events)."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
from transmvsnet_amd import TransMVSNet, synthetic
H, W, N = 1056, 1920, 11
dev = torch.device("cuda")
m = TransMVSNet().eval()
m.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=0, sharpen=100.0))
m = m.to(dev)
imgs = synthetic.synthetic_images(N, H, W).to(dev)
proj = synthetic.synthetic_cameras(N, H, W, seed=1)
dv = synthetic.synthetic_depth_values(1).to(dev)
ts = []
with torch.no_grad():
    for i in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = m.forward(imgs, proj, dv)
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1))
d = out["depth"]
assert torch.isfinite(d).all() and torch.isfinite(out["prob_volume"]).all()
assert float(d.min()) >= 425.0 and float(d.max()) <= 935.0
print(f"TnT {H}x{W} N={N}: forward {np.median(ts):.2f} ms ({1e3 / np.median(ts):.2f} depth maps/s), "
      f"depth range [{float(d.min()):.1f}, {float(d.max()):.1f}], peak mem {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB")
