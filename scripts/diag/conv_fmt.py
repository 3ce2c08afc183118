"""MIOpen conv2d timing at FeatureNet's full-resolution head shapes: NCHW vs channels_last (NHWC)."""
import torch, numpy as np, torch.nn.functional as F
dev = "cuda"
torch.backends.cudnn.benchmark = True
def timed(fn, n=10, w=3):
    ts = []
    for i in range(n + w):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize()
        if i >= w: ts.append(e0.elapsed_time(e1) * 1e3)
    return np.median(ts)
for (ci, co, k, h, w) in ((32, 27, 3, 864, 1152), (32, 32, 3, 864, 1152), (32, 27, 3, 432, 576), (8, 8, 3, 864, 1152), (16, 32, 5, 432, 576)):
    x = torch.randn(5, ci, h, w, device=dev)
    wt = torch.randn(co, ci, k, k, device=dev)
    b = torch.randn(co, device=dev)
    st = 2 if k == 5 else 1
    r = {}
    r["nchw"] = timed(lambda: F.conv2d(x, wt, b, stride=st, padding=k // 2))
    xc = x.to(memory_format=torch.channels_last); wc = wt.to(memory_format=torch.channels_last)
    r["nhwc"] = timed(lambda: F.conv2d(xc, wc, b, stride=st, padding=k // 2))
    y = F.conv2d(xc, wc, b, stride=st, padding=k // 2)
    print(f"{ci}->{co} k{k} {h}x{w}: " + " ".join(f"{kk} {v:.0f}us" for kk, v in r.items()),
          "out channels_last:", y.is_contiguous(memory_format=torch.channels_last), flush=True)
