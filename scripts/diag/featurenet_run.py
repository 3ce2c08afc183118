"""FeatureNet over the 5 DTU views (batched, as TransMVSNet.forward does), K times: the command
profiled by rocprofv3 to see where FeatureNet's time goes; prints the median HIP-event time of one forward
(FNET_SAVE=path also saves the outputs).
Usage: featurenet_run.py [K]"""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch
from transmvsnet_amd import TransMVSNet, synthetic
K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
H, W, N = 864, 1152, 5
dev = torch.device("cuda")
m = TransMVSNet().eval()
m.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=0, sharpen=100.0))
m = m.to(dev)
imgs = synthetic.synthetic_images(N, H, W).to(dev)
ts = []
with torch.no_grad():
    for i in range(K + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f = m.feature(imgs.reshape(N, 3, H, W))
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(e0.elapsed_time(e1))
ts.sort()
if os.environ.get("FNET_SAVE"):
    torch.save({k: v.cpu() for k, v in f.items()}, os.environ["FNET_SAVE"])
print(os.environ.get("TMVS_LIB_PATH") or "default", "side" if os.environ.get("TMVS_FNET_SIDE", "1") != "0" else "serial",
      f"FeatureNet {ts[len(ts) // 2]:.3f} ms (median of {K})",
      {k: tuple(v.shape) for k, v in f.items()})
