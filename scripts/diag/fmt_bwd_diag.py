"""Intermediate-by-intermediate check of the FMT layer backward against fp64 torch (diagnostic)."""
import sys
import torch
import torch.nn.functional as F
from transmvsnet_amd import ops
from transmvsnet_amd.train import _ENC_PARAMS, _pack_enc
from tests._util import golden_state_dict

L = int(sys.argv[1]) if len(sys.argv) > 1 else 27648
sd = golden_state_dict()
P = "FMT_with_pathway.FMT.layers.1."
p = [sd[P + n].to("cuda").contiguous() for n in _ENC_PARAMS]
g = torch.Generator().manual_seed(3)
src = torch.randn(L, 32, generator=g)
q = torch.randn(2 * L, 32, generator=g)
dmsg = torch.randn(2 * L, 32, generator=g)
D = torch.float64
wk, bk, wv, bv = (sd[P + n].to(D) for n in _ENC_PARAMS[2:6])
k64 = F.linear(src.to(D), wk, bk)
v64 = F.linear(src.to(D), wv, bv)
K = (F.elu(k64) + 1).view(L, 8, 4)
V = v64.view(L, 8, 4)
kv64 = torch.cat([torch.einsum("shd,shm->hmd", K, V).reshape(-1), K.sum(0).reshape(-1)])


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max())


kv = ops.fmt_kv(src.cuda()[None].contiguous(), _pack_enc(p))
print("kv", rel(kv[0], kv64))
k = ops.token_linear(src.cuda(), p[2], p[3])
v = ops.token_linear(src.cuda(), p[4], p[5])
print("k", rel(k, k64), "v", rel(v, v64))
# query side in fp64
qq = q.to(D).requires_grad_()
KVt = kv64.clone().requires_grad_()
Q = (F.elu(qq) + 1).view(2 * L, 8, 4)
KVm = KVt[:128].view(8, 4, 4)
Ks = KVt[128:].view(8, 4)
z = 1 / (torch.einsum("lhd,hd->lh", Q, Ks) + 1e-6)
msg = torch.einsum("lhd,hmd,lh->lhm", Q, KVm, z).reshape(2 * L, 32)
msg.backward(dmsg.to(D))
m = ops.linattn_fwd(q.cuda(), kv, 2 * L)
print("msg", rel(m, msg.detach()))
dq, dkv = ops.linattn_bwd_q(q.cuda(), dmsg.cuda(), kv, 2 * L)
print("dq", rel(dq, qq.grad), "dkv", rel(dkv[0], KVt.grad), "dKV part", rel(dkv[0, :128], KVt.grad[:128]),
      "dKs part", rel(dkv[0, 128:], KVt.grad[128:]))
kk = k64.clone().requires_grad_()
vv = v64.clone().requires_grad_()
K2 = (F.elu(kk) + 1).view(L, 8, 4)
kvr = torch.cat([torch.einsum("shd,shm->hmd", K2, vv.view(L, 8, 4)).reshape(-1), K2.sum(0).reshape(-1)])
kvr.backward(KVt.grad)
dk, dv = ops.linattn_bwd_kv(k, v, dkv, L)
print("dk", rel(dk, kk.grad), "dv", rel(dv, vv.grad))
dk2, dv2 = ops.linattn_bwd_kv(k, v, KVt.grad.float().cuda()[None].contiguous(), L)
print("dk from exact dkv", rel(dk2, kk.grad), "dv", rel(dv2, vv.grad))
