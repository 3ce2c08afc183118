"""Depth maps/s on one MI355X for the BASELINE.json configurations' shapes: hot path (forward_features
from resident features) and the whole forward from images. C2 = DTU 864x1152 N=5 (the bench), C3
shape = DTU N=11 (BASELINE runs it view-sharded on 2 GPUs; here one GPU), C4 shape = Tanks&Temples
1056x1920 N=11 (BASELINE: 8 GPUs view-parallel; here one GPU). HIP events, median of 5 after 2."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import json
import numpy as np, torch
from transmvsnet_amd import TransMVSNet, synthetic

dev = torch.device("cuda")
m = TransMVSNet().eval()
m.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=0, sharpen=100.0))
m = m.to(dev)


def timed(fn, n=5, w=2):
    ts = []
    for i in range(n + w):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i >= w:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


res = {}
for name, (H, W, N) in {"C2_dtu_n5": (864, 1152, 5), "C3_dtu_n11": (864, 1152, 11),
                        "C4_tnt_n11": (1056, 1920, 11)}.items():
    imgs = synthetic.synthetic_images(N, H, W).to(dev)
    proj = synthetic.synthetic_cameras(N, H, W, seed=1)
    dv = synthetic.synthetic_depth_values(1).to(dev)
    with torch.no_grad():
        f = m.feature(imgs.reshape(N, 3, H, W))
        feats = {k: v.reshape(1, N, *v.shape[1:]).contiguous() for k, v in f.items()}
        t_hot = timed(lambda: m.forward_features(feats, proj, dv, (H, W)))
        t_all = timed(lambda: m.forward(imgs, proj, dv))
    res[name] = {"H": H, "W": W, "N": N, "hot_path_ms": round(t_hot, 3), "hot_path_depth_maps_per_s": round(1e3 / t_hot, 2),
                 "forward_ms": round(t_all, 3), "forward_depth_maps_per_s": round(1e3 / t_all, 2)}
    print(name, res[name], flush=True)
    del imgs, f, feats
    torch.cuda.empty_cache()
print(json.dumps(res))
