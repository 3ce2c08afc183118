"""FMT launches alone at the C2 stage-1 shape (5 views, 216x288 tokens), HIP-event medians.

    python scripts/diag/fmt_time.py [REPS]          (TMVS_LIB_PATH selects a library variant)
Prints the per-launch medians of tmvs_fmt_kv (5 views / 1 view), tmvs_fmt_apply (5 / 4 views) and the
whole tmvs_fmt_forward, and a bit-level digest of the FMT output (A/B builds must print the same digest).
"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from transmvsnet_amd import TransMVSNet, ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = TransMVSNet().eval()
# non-trivial encoder weights: the reference's xavier init, re-drawn per layer with a fixed seed
g = torch.Generator().manual_seed(1)
with torch.no_grad():
    for p in m.FMT_with_pathway.parameters():
        p.copy_(torch.randn(p.shape, generator=g) * (0.3 if p.dim() > 1 else 0.05))
m.invalidate()
prep = m._prepared(dev)
nv, h, w = 5, 216, 288
s1 = torch.randn(nv, 32, h, w, device=dev)
pe = m._pe_slice(h, w, dev)
enc = prep["enc"]


def med(fn):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


tok = ops.fmt_forward(s1, pe, enc)
torch.cuda.synchronize()
digest = hashlib.sha1(tok.cpu().numpy().tobytes()).hexdigest()[:16]
x5 = tok.clone()
kv5 = ops.fmt_kv(x5, enc[0])
kv1 = ops.fmt_kv(x5[:1], enc[1])
kvd = hashlib.sha1(torch.cat([kv5.flatten(), kv1.flatten()]).cpu().numpy().tobytes()).hexdigest()[:16]
res = {}
res["kv5"] = med(lambda: ops.fmt_kv(x5, enc[0], out=kv5))
res["kv1"] = med(lambda: ops.fmt_kv(x5[:1], enc[1], out=kv1))
x5b = tok.clone()
res["apply5"] = med(lambda: ops.fmt_apply(x5b, kv5, enc[0]))
x4 = tok[1:].clone()
res["apply4"] = med(lambda: ops.fmt_apply(x4, kv1, enc[1], shared_kv=True))
out = torch.empty_like(tok)
res["forward"] = med(lambda: ops.fmt_forward(s1, pe, enc, tokens=out))
side = torch.cuda.Stream(dev)
res["split"] = med(lambda: ops.fmt_forward(s1, pe, enc, tokens=out, side_stream=side))
torch.cuda.synchronize()
assert torch.equal(out, tok), "split FMT tokens differ"
# graph-replayed (launch overhead out): one capture per form
for name, kw in (("forward_graph", {}), ("split_graph", {"side_stream": side})):
    ops.fmt_forward(s1, pe, enc, tokens=out, **kw)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        ops.fmt_forward(s1, pe, enc, tokens=out, **kw)
    res[name] = med(gr.replay)
    torch.cuda.synchronize()
    assert torch.equal(out, tok), f"{name} tokens differ"
print(f"fmt {os.environ.get('TMVS_LIB_PATH', 'default')} tpw={os.environ.get('TMVS_APPLY_TPW', '-')}: "
      + " ".join(f"{k} {v:.1f}us" for k, v in res.items()) + f" | tokens {digest} kv {kvd}", flush=True)
