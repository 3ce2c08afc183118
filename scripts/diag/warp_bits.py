"""Which step of homo_warping does the GPU compute differently from torch-CPU? (diagnostic)

Stage-3-like case (C=8, D=8, 864x1152, per-pixel hypotheses). Compares, bit for bit, torch's
intermediates (rot_xyz, proj_xyz, normalised grid, grid_sample output) with float32 emulations of
candidate op orders (numpy; fma emulated in float64, exact for fp32 operands), and the GPU seam
tmvs_homo_warping's output with torch's. Runs on the CPU alone when no GPU is present.
"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch
import torch.nn.functional as F

from oracle import transmvs_ref as oracle
from transmvsnet_amd import synthetic

torch.set_num_threads(int(os.environ.get("THREADS", "16")))
H, W, C, D = 864, 1152, 8, 8
ROWS = int(os.environ.get("ROWS", "64"))  # evaluate this many reference rows (all columns)
f32 = np.float32


def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def frac_eq(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float((a == b).mean()), float(np.abs(a.astype(np.float64) - b.astype(np.float64)).max())


proj = synthetic.synthetic_cameras(2, H, W, seed=1)["stage3"]
g = torch.Generator().manual_seed(5)
src = torch.randn(1, C, H, W, generator=g)
hyp = (600.0 + 40.0 * torch.rand(1, D, H, W, generator=g)).contiguous()
src_p, ref_p = oracle.compose_proj(proj[:, 1]), oracle.compose_proj(proj[:, 0])

with torch.no_grad():
    P = torch.matmul(src_p, torch.inverse(ref_p))
    rot, trans = P[:, :3, :3], P[:, :3, 3:4]
    y, x = torch.meshgrid([torch.arange(0, H, dtype=torch.float32), torch.arange(0, W, dtype=torch.float32)],
                          indexing="ij")
    y, x = y.contiguous().view(H * W), x.contiguous().view(H * W)
    xyz = torch.stack((x, y, torch.ones_like(x))).unsqueeze(0)
    rot_xyz = torch.matmul(rot, xyz)
    rdx = rot_xyz.unsqueeze(2).repeat(1, 1, D, 1) * hyp.view(1, 1, D, -1)
    pxyz = rdx + trans.view(1, 3, 1, 1)
    pxy = pxyz[:, :2] / pxyz[:, 2:3]
    xn = pxy[:, 0] / ((W - 1) / 2) - 1
    yn = pxy[:, 1] / ((H - 1) / 2) - 1
    grid = oracle.warp_grid(src_p, ref_p, hyp, H, W)
    out = F.grid_sample(src, grid, mode="bilinear", padding_mode="zeros", align_corners=True).view(1, C, D, H, W)

R = rot[0].numpy()
T = trans[0, :, 0].numpy()
xs, ys = x.numpy(), y.numpy()
rx_t = rot_xyz[0].numpy()
cands = {
    "fma(r1,y,r0*x)+r2": lambda i: fma(R[i, 1], ys, R[i, 0] * xs) + R[i, 2],
    "(r0*x+r1*y)+r2": lambda i: (R[i, 0] * xs + R[i, 1] * ys) + R[i, 2],
    "fma(r0,x,fma(r1,y,r2))": lambda i: fma(R[i, 0], xs, fma(R[i, 1], ys, np.full_like(xs, R[i, 2]))),
    "fma(r2,1,fma(r1,y,fma(r0,x,0)))": lambda i: fma(np.full_like(xs, R[i, 2]), np.ones_like(xs),
                                                     fma(R[i, 1], ys, fma(R[i, 0], xs, np.zeros_like(xs)))),
    "r0*x+(r1*y+r2)": lambda i: R[i, 0] * xs + (R[i, 1] * ys + R[i, 2]),
    "fma(r0,x,r1*y)+r2": lambda i: fma(R[i, 0], xs, R[i, 1] * ys) + R[i, 2],
}
print("rot_xyz (matmul [3,3]x[3,HW]):")
for name, fn in cands.items():
    res = [frac_eq(fn(i), rx_t[i]) for i in range(3)]
    print(f"  {name:36s} exact {[round(r[0], 5) for r in res]}  maxdiff {[f'{r[1]:.1e}' for r in res]}")

hyp_np = hyp[0].numpy().reshape(D, -1)
emx = rx_t[:, None, :] * hyp_np[None] + T[:, None, None]  # uses torch's rot_xyz
print("proj_xyz from torch rot_xyz:", frac_eq(emx, pxyz[0].numpy()))
ex_xn = (emx[0] / emx[2]) / f32((W - 1) / 2) - f32(1)
print("x normalised from torch proj_xyz:", frac_eq(ex_xn, xn[0].numpy()))
gx = grid[0, :, :, 0].numpy().reshape(D, -1)
print("grid x vs normalised x:", frac_eq(gx, xn[0].numpy()))

# grid_sample restated from the torch grid (GPU formula)
n = ROWS * W
gxs, gys = grid[0, :, :, 0].numpy().reshape(D, H * W)[:, :n], grid[0, :, :, 1].numpy().reshape(D, H * W)[:, :n]
ix = (gxs + f32(1)) * f32((W - 1) / 2)
iy = (gys + f32(1)) * f32((H - 1) / 2)
x0, y0 = np.floor(ix), np.floor(iy)
we, nn_ = ix - x0, iy - y0
ea, s = f32(1) - we, f32(1) - nn_
wnw, wne, wsw, wse = s * ea, s * we, nn_ * ea, nn_ * we
S = src[0].numpy()


def tap(xx, yy):
    ok = (xx >= 0) & (xx <= W - 1) & (yy >= 0) & (yy <= H - 1)
    xi = np.where(ok, xx, 0).astype(np.int64)
    yi = np.where(ok, yy, 0).astype(np.int64)
    return np.where(ok[None], S[:, yi, xi], f32(0))


a, b, c, d = tap(x0, y0), tap(x0 + 1, y0), tap(x0, y0 + 1), tap(x0 + 1, y0 + 1)
ref_out = out[0].numpy().reshape(C, D, H * W)[:, :, :n]
variants = {
    "fma(se,fma(sw,fma(ne,nw*)))": fma(d, wse, fma(c, wsw, fma(b, wne, a * wnw))),
    "((nw+ne)+sw)+se no fma": ((a * wnw + b * wne) + c * wsw) + d * wse,
    "fma chain from nw": fma(d, wse, fma(c, wsw, fma(b, wne, a * wnw))),
}
print("grid_sample output from the torch grid:")
for name, v in variants.items():
    print(f"  {name:30s}", frac_eq(v, ref_out))

if torch.cuda.is_available():
    from transmvsnet_amd import ops
    og = ops.homo_warping(src.cuda(), src_p, ref_p, hyp.cuda()).cpu()
    print("GPU tmvs_homo_warping vs torch:", frac_eq(og.numpy(), out.numpy()))
    bad = np.argwhere(og.numpy() != out.numpy())[:5]
    for (bb, cc, dd, yy, xx) in bad:
        p = yy * W + xx
        print(f"  c{cc} d{dd} y{yy} x{xx}: gpu {og[bb, cc, dd, yy, xx].item():.9g} torch {out[bb, cc, dd, yy, xx].item():.9g}"
              f" grid ({grid[0, dd * H + yy, xx, 0].item():.9g}, {grid[0, dd * H + yy, xx, 1].item():.9g})")
