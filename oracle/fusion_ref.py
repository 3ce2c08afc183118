"""CPU restatement of the reference's depth-map fusion (gipuma/fusibile) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module; the
product path is transmvsnet_amd/fusion.py + the HIP kernel tmvs_fusibile (csrc/fusion.hip).

Follows gipuma/fusibile/fusibile.cu:89-173 (the `fusibile` kernel), :206-229 (copy_pc_to_host),
:231-286 (the per-camera loop), main.cpp:126-148 (RGBA -> (B, G, R, 425 + 512 * alpha)) and
cameraGeometryUtils.h:100-162 (camera parameters). Evaluated in float64, so it is the exact value
of the reference's float formulas; the HIP kernel is compared to it with stated tolerances.

Parity unpinned: fusibile needs CUDA and OpenCV (absent here), and the reference ships no fused
point clouds. Two pieces of reference behaviour are reproduced on purpose:
  * the point buffer is allocated and zeroed ONCE (main.cpp:140-141) and each camera's kernel only
    overwrites the pixels it fuses, so copy_pc_to_host (fusibile.cu:206-229) re-emits every earlier
    camera's surviving pixel that this camera did not overwrite;
  * `operator+` / `operator/` on float4 (fusibile.cu:18-31) zero the .w component.
Texture sampling (main.cpp:30-66: cudaFilterModeLinear, unnormalised coordinates, which CUDA
clamps regardless of the requested wrap mode) is emulated as documented for CUDA: texel centres
at i + 0.5, fractional weights with 8 fractional bits (rounded to nearest here).
"""
from __future__ import annotations

import numpy as np

DEPTH_FLOOR = 425.001  # fusibile.cu:116, 141


def tex_linear(img, x, y):
    """tex2D<float4> with linear filtering at unnormalised (x, y) (already including the +0.5):
    img [H, W, 4]; x, y arrays. Clamp addressing, 8-bit fractions."""
    h, w = img.shape[:2]
    xb = x.astype(np.float64) - 0.5
    yb = y.astype(np.float64) - 0.5
    i0 = np.floor(xb)
    j0 = np.floor(yb)
    a = np.round((xb - i0) * 256.0) / 256.0
    b = np.round((yb - j0) * 256.0) / 256.0
    i0 = i0.astype(np.int64)
    j0 = j0.astype(np.int64)
    i1 = np.clip(i0 + 1, 0, w - 1)
    j1 = np.clip(j0 + 1, 0, h - 1)
    i0 = np.clip(i0, 0, w - 1)
    j0 = np.clip(j0, 0, h - 1)
    t = img.astype(np.float64)
    a = a[..., None]
    b = b[..., None]
    return ((1 - a) * (1 - b) * t[j0, i0] + a * (1 - b) * t[j0, i1] + (1 - a) * b * t[j1, i0]
            + a * b * t[j1, i1])


def get_3dpoint(cam, px, py, depth):
    """get_3dpoint_cu (fusibile.cu:54-68): RK_inv @ (d*x - P34.x, d*y - P34.y, d - P34.z)."""
    c34 = cam["P"][:, 3]
    pt = np.stack([depth * px - c34[0], depth * py - c34[1], depth - c34[2]], -1)
    return pt @ cam["RK_inv"].T


def project(cam, X):
    """project_on_camera (fusibile.cu:75-84): (x/z, y/z, z) of P @ [X, 1]."""
    t = X @ cam["P"][:, :3].T + cam["P"][:, 3]
    return t[..., 0] / t[..., 2], t[..., 1] / t[..., 2], t[..., 2]


def fusibile_ref(rgbd, cams, ref, consistent_threshold=3, depth_threshold=0.25):
    """The fusibile kernel for one reference camera (fusibile.cu:89-173).

    rgbd [V, H, W, 4] float32 (B, G, R, depth); cams: list of dicts (P [3,4], RK_inv [3,3], C4 [3],
    fx). Returns (written [H, W] bool, coord [H, W, 3], texture [H, W, 3]) for the written pixels."""
    v, h, w, _ = rgbd.shape
    ys, xs = np.mgrid[0:h, 0:w]
    ys = ys.astype(np.float64)
    xs = xs.astype(np.float64)
    ref_t = rgbd[ref].astype(np.float64)
    depth = ref_t[..., 3]
    alive = depth > DEPTH_FLOOR
    X = get_3dpoint(cams[ref], xs, ys, depth)
    sum_x = X.copy()
    sum_t = ref_t[..., :3].copy()
    count = np.zeros((h, w), np.int64)
    f = cams[ref]["fx"]
    for i in range(v):
        if i == ref:
            continue
        act = alive & (count < 2 * consistent_threshold)
        px, py, d = project(cams[i], X)
        act &= ~((px < 0) | (px >= w) | (py < 0) | (py >= h))
        act &= np.isfinite(px) & np.isfinite(py)
        pxs = np.where(act, px, 0.0)
        pys = np.where(act, py, 0.0)
        tt = tex_linear(rgbd[i], pxs + 0.5, pys + 0.5)
        act &= tt[..., 3] > DEPTH_FLOOR
        base = np.linalg.norm(np.asarray(cams[ref]["C4"], np.float64) - np.asarray(cams[i]["C4"], np.float64))
        with np.errstate(divide="ignore", invalid="ignore"):
            dd = f * base / d
            td = f * base / tt[..., 3]
        act &= np.abs(dd - td) < depth_threshold
        tx = get_3dpoint(cams[i], np.floor(pxs), np.floor(pys), tt[..., 3])
        sum_x += np.where(act[..., None], tx, 0.0)
        sum_t += np.where(act[..., None], tt[..., :3], 0.0)
        count += act
    written = alive & (count >= consistent_threshold)
    n1 = (count + 1.0)[..., None]
    return written, sum_x / n1, sum_t / n1


def fuse_ref(rgbd, cams, consistent_threshold=3, depth_threshold=0.25):
    """run_fusibile's camera loop with the persistent point buffer and copy_pc_to_host
    (fusibile.cu:206-229, 265-271): returns the concatenated (coord [N,3], texture [N,3])."""
    v, h, w, _ = rgbd.shape
    buf_x = np.zeros((h, w, 3))
    buf_t = np.zeros((h, w, 3))
    out_x, out_t = [], []
    for cam in range(v):
        wr, cx, ct = fusibile_ref(rgbd, cams, cam, consistent_threshold, depth_threshold)
        buf_x[wr] = cx[wr]
        buf_t[wr] = ct[wr]
        keep = (buf_x[..., 0] != 0) & (buf_x[..., 1] != 0) & (buf_x[..., 2] != 0)
        out_x.append(buf_x[keep])
        out_t.append(buf_t[keep])
    return np.concatenate(out_x), np.concatenate(out_t)
