"""Input side: the reference's dataset readers, so real DTU / Tanks&Temples
scans can be fed to ``TransMVSNet.forward`` instead of synthetic tensors.

  read_pfm / save_pfm          datasets/data_io.py:6-78 (pinned byte-for-byte: tests/golden/pfm.npz)
  read_pair_file               datasets/general_eval.py:41-56 (view selection, fill to nviews)
  read_cam_file                datasets/general_eval.py:67-97 (DTU: intrinsics / 4, depth range);
                               tnt=True: datasets/tnt_eval.py:69-83
  read_img                     datasets/general_eval.py:99-103 (PIL, / 255)
  scale_mvs_input              datasets/general_eval.py:106-124 (resize to a multiple of 32)
  load_sample                  datasets/general_eval.py:126-210 (imgs, 3-stage proj_matrix, depth_values)
  read_pair_file(pad=False)    datasets/tnt_eval.py:44-59 (no filling: the sample shrinks instead)
  load_sample_tnt              datasets/tnt_eval.py:120-210 (cams_1/, per-scan image_sizes caps, nviews
                               shrunk to 1 + #sources, np.arange(dmin, dint*nd + dmin, dint), optional
                               inverse-depth hypotheses, the dataset-wide fixed resolution)

Host-side, as in the reference (its DataLoader workers). The reference resizes with
cv2.resize(INTER_LINEAR) -- absent here; ``resize_bilinear`` restates OpenCV's float path
(half-pixel centres, edge-clamped neighbours); that piece is parity-unpinned.
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np


# ------------------------------------------------------------------ PFM (datasets/data_io.py)
def read_pfm(filename):
    """data_io.read_pfm: returns (data flipped to top-down [H,W] or [H,W,3] float32, scale)."""
    with open(filename, "rb") as f:
        header = f.readline().decode("utf-8").rstrip()
        if header not in ("PF", "Pf"):
            raise Exception("Not a PFM file.")
        colour = header == "PF"
        m = re.match(r"^(\d+)\s(\d+)\s$", f.readline().decode("utf-8"))
        if not m:
            raise Exception("Malformed PFM header.")
        width, height = map(int, m.groups())
        scale = float(f.readline().rstrip())
        endian = "<" if scale < 0 else ">"
        scale = abs(scale)
        data = np.fromfile(f, endian + "f")
    data = np.reshape(data, (height, width, 3) if colour else (height, width))
    return np.flipud(data), scale


def save_pfm(filename, image, scale=1):
    """data_io.save_pfm: 'PF'/'Pf', 'W H', signed scale (negative = little endian), bottom-up rows."""
    image = np.flipud(image)
    if image.dtype.name != "float32":
        raise Exception("Image dtype must be float32.")
    if image.ndim == 3 and image.shape[2] == 3:
        colour = True
    elif image.ndim == 2 or (image.ndim == 3 and image.shape[2] == 1):
        colour = False
    else:
        raise Exception("Image must have H x W x 3, H x W x 1 or H x W dimensions.")
    endian = image.dtype.byteorder
    if endian == "<" or (endian == "=" and sys.byteorder == "little"):
        scale = -scale
    with open(filename, "wb") as f:
        f.write(b"PF\n" if colour else b"Pf\n")
        f.write("{} {}\n".format(image.shape[1], image.shape[0]).encode("utf-8"))
        f.write(("%f\n" % scale).encode("utf-8"))
        image.tofile(f)


# ------------------------------------------------------------------ scan files (general_eval.py)
def read_pair_file(filename, nviews=5, pad=True):
    """general_eval.build_list for one scan: [(ref_view, [src views...])]; views without sources are
    dropped, fewer than nviews sources are filled with the first source (:47-56). pad=False is
    tnt_eval.build_list (:44-59): no filling (load_sample_tnt shrinks the view count instead)."""
    metas = []
    with open(filename) as f:
        n = int(f.readline())
        for _ in range(n):
            ref = int(f.readline().rstrip())
            src = [int(x) for x in f.readline().rstrip().split()[1::2]]
            if len(src) > 0:
                if pad and len(src) < nviews:
                    src += [src[0]] * (nviews - len(src))
                metas.append((ref, src))
    return metas


def read_cam_file(filename, ndepths=192, interval_scale=1.0, tnt=False):
    """general_eval.read_cam_file (:67-97): extrinsic 4x4 (lines 1-4), intrinsic 3x3 (lines 7-9)
    with fx, fy, cx, cy divided by 4, line 11 = depth_min, depth_interval[, num_depth]. With tnt=True
    tnt_eval.read_cam_file (:69-83): line 11 = depth_min, depth_max. Returns (intrinsics,
    extrinsics, depth_min, depth_interval[, depth_max])."""
    with open(filename) as f:
        lines = [ln.rstrip() for ln in f.readlines()]
    extrinsics = np.array(" ".join(lines[1:5]).split(), np.float32).reshape(4, 4)
    intrinsics = np.array(" ".join(lines[7:10]).split(), np.float32).reshape(3, 3)
    intrinsics[:2, :] /= 4.0
    fields = lines[11].split()
    depth_min = float(fields[0])
    if tnt:
        depth_max = float(fields[1])
        return intrinsics, extrinsics, depth_min, float((depth_max - depth_min) / ndepths), depth_max
    depth_interval = float(fields[1])
    if len(fields) >= 3:
        depth_max = depth_min + int(float(fields[2])) * depth_interval
        depth_interval = (depth_max - depth_min) / ndepths
    return intrinsics, extrinsics, depth_min, depth_interval * interval_scale


def read_img(filename):
    """general_eval.read_img: PIL image -> float32 in [0, 1]."""
    from PIL import Image
    return np.array(Image.open(filename), dtype=np.float32) / 255.0


def resize_bilinear(img, new_w, new_h):
    """cv2.resize(img, (new_w, new_h)) with INTER_LINEAR for float images: source coordinate
    (x + 0.5) * (w / new_w) - 0.5, neighbours clamped to the image, separable lerp in float32."""
    img = np.asarray(img, np.float32)
    h, w = img.shape[:2]

    def axis(n_out, n_in):
        f = (np.arange(n_out, dtype=np.float64) + 0.5) * (n_in / n_out) - 0.5
        i0 = np.floor(f)
        t = (f - i0).astype(np.float32)
        i0 = i0.astype(np.int64)
        t = np.where(i0 < 0, np.float32(0), t)
        i0 = np.clip(i0, 0, n_in - 1)
        t = np.where(i0 >= n_in - 1, np.float32(0), t)
        return i0, np.minimum(i0 + 1, n_in - 1), t.astype(np.float32)

    x0, x1, tx = axis(int(new_w), w)
    y0, y1, ty = axis(int(new_h), h)
    bx = tx.reshape((1, -1) + (1,) * (img.ndim - 2))
    by = ty.reshape((-1,) + (1,) * (img.ndim - 1))
    rows = img[:, x0] * (np.float32(1) - bx) + img[:, x1] * bx  # horizontal pass, then vertical
    return (rows[y0] * (np.float32(1) - by) + rows[y1] * by).astype(np.float32)


def scale_mvs_input(img, intrinsics, max_w, max_h, base=32):
    """general_eval.scale_mvs_input (:106-124): fit into (max_w, max_h) keeping the aspect ratio,
    round both sides down to a multiple of `base`, rescale the intrinsics rows accordingly."""
    h, w = img.shape[:2]
    if h > max_h or w > max_w:
        scale = 1.0 * max_h / h
        if scale * w > max_w:
            scale = 1.0 * max_w / w
        new_w, new_h = scale * w // base * base, scale * h // base * base
    else:
        new_w, new_h = 1.0 * w // base * base, 1.0 * h // base * base
    intrinsics = intrinsics.copy()
    intrinsics[0, :] *= 1.0 * new_w / w
    intrinsics[1, :] *= 1.0 * new_h / h
    return resize_bilinear(img, int(new_w), int(new_h)), intrinsics


def _stack_sample(imgs, projs, depth_values, scan, ref_view):
    imgs = np.stack(imgs).transpose(0, 3, 1, 2)
    proj = np.stack(projs)
    s2, s3 = proj.copy(), proj.copy()
    s2[:, 1, :2, :] = proj[:, 1, :2, :] * 2
    s3[:, 1, :2, :] = proj[:, 1, :2, :] * 4
    return {"imgs": imgs, "proj_matrix": {"stage1": proj, "stage2": s2, "stage3": s3},
            "depth_values": depth_values, "filename": scan + "/{}/" + "{:0>8}".format(ref_view) + "{}"}


# Tanks&Temples image sizes (datasets/tnt_eval.py:24-37): the per-scan (max_w, max_h) of scale_mvs_input
TNT_IMAGE_SIZES = {"Family": (1920, 1080), "Francis": (1920, 1080), "Horse": (1920, 1080),
                   "Lighthouse": (2048, 1080), "M60": (2048, 1080), "Panther": (2048, 1080),
                   "Playground": (1920, 1080), "Train": (1920, 1080), "Auditorium": (1920, 1080),
                   "Ballroom": (1920, 1080), "Courtroom": (1920, 1080), "Museum": (1920, 1080),
                   "Palace": (1920, 1080), "Temple": (1920, 1080)}


def load_sample_tnt(datapath, scan, ref_view, src_views, nviews=11, ndepths=192, interval_scale=1.0,
                    inverse_depth=False, fixed_hw=None, image_size=None):
    """tnt_eval.MVSDataset.__getitem__ (:120-210) for one (scan, ref, srcs).

    nviews shrinks to 1 + len(src_views) when there are fewer sources (:125-126). Images come from
    {scan}/images/, cameras from {scan}/cams_1/ (read_cam_file(tnt=True): depth_min, depth_max on line
    11); each image is fitted into the scan's TNT_IMAGE_SIZES (or `image_size` = (max_w, max_h) for a
    scan outside the table). The reference fixes ONE resolution for the whole dataset from the first
    image it ever loads (fix_res, :137-141): pass that (h, w) as `fixed_hw` to reproduce it across
    samples; by default this sample's reference image sets it. Returns the dict of load_sample plus
    "fixed_hw"."""
    nviews = min(nviews, len(src_views) + 1)
    view_ids = [ref_view] + list(src_views[:nviews - 1])
    max_w, max_h = image_size if image_size is not None else TNT_IMAGE_SIZES[scan]
    imgs, projs, depth_values = [], [], None
    s_h, s_w = fixed_hw if fixed_hw is not None else (None, None)
    for i, vid in enumerate(view_ids):
        img = read_img(os.path.join(datapath, "{}/images/{:0>8}.jpg".format(scan, vid)))
        intr, extr, dmin, dint, dmax = read_cam_file(
            os.path.join(datapath, "{}/cams_1/{:0>8}_cam.txt".format(scan, vid)), ndepths, tnt=True)
        img, intr = scale_mvs_input(img, intr, max_w, max_h)
        if s_h is None:
            s_h, s_w = img.shape[:2]
        c_h, c_w = img.shape[:2]
        if (c_h, c_w) != (s_h, s_w):
            img = resize_bilinear(img, s_w, s_h)
            intr[0, :] *= 1.0 * s_w / c_w
            intr[1, :] *= 1.0 * s_h / c_h
        imgs.append(img)
        p = np.zeros((2, 4, 4), np.float32)
        p[0] = extr
        p[1, :3, :3] = intr
        projs.append(p)
        if i == 0:
            if not inverse_depth:
                depth_values = np.arange(dmin, dint * ndepths + dmin, dint, dtype=np.float32)
            else:  # tnt_eval.py:181-185
                depth_end = dmax - dint / interval_scale
                depth_values = (1.0 / np.linspace(1.0 / depth_end, 1.0 / dmin, ndepths, endpoint=False)).astype(
                    np.float32)
    out = _stack_sample(imgs, projs, depth_values, scan, ref_view)
    out["fixed_hw"] = (s_h, s_w)
    return out


def load_sample(datapath, scan, ref_view, src_views, nviews=5, ndepths=192, interval_scale=1.0, max_h=864,
                max_w=1152):
    """general_eval.MVSDataset.__getitem__ (:126-210) for one (scan, ref, srcs): imgs [N,3,H,W],
    proj_matrix {stage1..3: [N,2,4,4]} (stage 2/3 intrinsics rows 0-1 x2 / x4), depth_values [D]."""
    view_ids = [ref_view] + list(src_views[:nviews - 1])
    imgs, projs, depth_values = [], [], None
    s_h = s_w = None
    for i, vid in enumerate(view_ids):
        img_fn = os.path.join(datapath, "{}/images_post/{:0>8}.jpg".format(scan, vid))
        if not os.path.exists(img_fn):
            img_fn = os.path.join(datapath, "{}/images/{:0>8}.jpg".format(scan, vid))
        cam_fn = os.path.join(datapath, "{}/cams/{:0>8}_cam.txt".format(scan, vid))
        img = read_img(img_fn)
        intr, extr, dmin, dint = read_cam_file(cam_fn, ndepths, interval_scale)
        img, intr = scale_mvs_input(img, intr, max_w, max_h)
        if i == 0:
            s_h, s_w = img.shape[:2]
        c_h, c_w = img.shape[:2]
        if (c_h, c_w) != (s_h, s_w):
            intr[0, :] *= 1.0 * s_w / c_w
            intr[1, :] *= 1.0 * s_h / c_h
            img = resize_bilinear(img, s_w, s_h)
        imgs.append(img)
        p = np.zeros((2, 4, 4), np.float32)
        p[0] = extr
        p[1, :3, :3] = intr
        projs.append(p)
        if i == 0:
            depth_values = np.arange(dmin, dint * (ndepths - 0.5) + dmin, dint, dtype=np.float32)
    return _stack_sample(imgs, projs, depth_values, scan, view_ids[0])
