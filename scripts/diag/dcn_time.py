"""Time tmvs_deform_conv2d at the FeatureNet head sizes (5 DTU views batched), offsets ~N(0, 1.5) px.
HIP events on the current stream, median of 10 after 3 warm-ups. Variant via TMVS_DCN_* env.
DCN_FUSED=1 times tmvs_dcn_fused; with DCN_SAVE=path / DCN_COMPARE=path its outputs are saved / compared bit for bit."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
from transmvsnet_amd import ops
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(0)
res = []
outs = {}
CFGS = ((864, 1152, 32), (864, 1152, 8), (432, 576, 32), (432, 576, 16), (216, 288, 32))
only = os.environ.get("DCN_ONLY")
for (h, w, co) in ([CFGS[int(only)]] if only else CFGS):
    x = torch.randn(5, h, w, 32, generator=g).to(dev)
    om = torch.randn(5, 27, h, w, generator=g)
    om[:, :18] *= float(os.environ.get("DCN_OFFSET_STD", "1.5"))
    om = om.to(dev)
    wp = ops.deform_conv2d_pack(torch.randn(co, 32, 3, 3, generator=g) * 0.06).to(dev)
    bias = torch.zeros(co, device=dev)
    # fused: conv_offset_mask weights scaled so offsets have about DCN_OFFSET_STD pixels
    wom = ops.deform_conv2d_pack(torch.randn(27, 32, 3, 3, generator=g) * float(os.environ.get("DCN_OFFSET_STD", "1.5")) / 17).to(dev)
    bom = torch.zeros(27, device=dev)
    fused = os.environ.get("DCN_FUSED") is not None
    ts = []
    for i in range(13):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if fused:
            ops.dcn_fused(x, wom, bom, wp, bias, co, want_nchw=False, want_nhwc=True)
        else:
            ops.deform_conv2d(x, om, wp, bias, co, want_nhwc=True)
        e1.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1) * 1e3)
    tag = ""
    if fused and (os.environ.get("DCN_SAVE") or os.environ.get("DCN_COMPARE")):
        y = ops.dcn_fused(x, wom, bom, wp, bias, co, want_nchw=False, want_nhwc=True)[1].cpu()
        key = f"{h}x{w}x{co}"
        if os.environ.get("DCN_SAVE"):
            outs[key] = y
        else:
            ref = torch.load(os.environ["DCN_COMPARE"], weights_only=True)[key]
            tag = " ==" if torch.equal(ref, y) else f" DIFF {(ref - y).abs().max().item():.2e}"
    res.append(f"{h}x{w}->{co}: {np.median(ts):.1f} us{tag}")
print(os.environ.get("TMVS_DCN_TAG", "default"), "offset std", os.environ.get("DCN_OFFSET_STD", "1.5"), " | ".join(res))
if os.environ.get("DCN_SAVE"):
    torch.save(outs, os.environ["DCN_SAVE"])
