"""The C-ABI boundary without a GPU: the library builds for gfx950, loads, exports every
function include/transmvs.h declares with the argument count the ctypes binding uses, and the
host-only entry points behave (version, status strings, BN fold, argument validation).
Also: the product path refuses CPU tensors (no fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from transmvsnet_amd import _lib, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "transmvs.h")


def _declarations():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    decls = {}
    for m in re.finditer(r"\b(?:int|size_t|const\s+char\s*\*)\s*\*?\s*(tmvs_\w+)\s*\(([^)]*)\)\s*;", src):
        args = m.group(2).strip()
        n = 0 if args in ("", "void") else args.count(",") + 1
        decls[m.group(1)] = n
    return decls


@pytest.fixture(scope="module")
def lib():
    build.build()
    return _lib.load()


def test_header_declarations_match_binding():
    decls = _declarations()
    assert len(decls) >= 20
    assert set(decls) == set(_lib.SIGNATURES), set(decls) ^ set(_lib.SIGNATURES)
    for name, n in decls.items():
        assert len(_lib.SIGNATURES[name][1]) == n, name


def test_library_exports_every_symbol(lib):
    for name in _declarations():
        assert hasattr(lib, name), name
    assert lib.tmvs_abi_version() == _lib.ABI_VERSION


def test_header_constants_match_binding():
    src = open(HEADER).read()
    consts = dict(re.findall(r"#define\s+(TMVS_\w+)\s+(-?\d+)", src))
    assert int(consts["TMVS_ABI_VERSION"]) == _lib.ABI_VERSION
    assert int(consts["TMVS_PW_NPARAMS"]) == _lib.PW_NPARAMS
    assert int(consts["TMVS_ENC_NPARAMS"]) == _lib.ENC_NPARAMS
    assert int(consts["TMVS_KV_NFLOATS"]) == _lib.KV_NFLOATS
    assert int(consts["TMVS_WARP_PARTIAL"]) == _lib.WARP_PARTIAL
    assert int(consts["TMVS_WARP_ROT_PLAIN"]) == _lib.WARP_ROT_PLAIN


def test_status_strings(lib):
    for code in (0, -1, -2, -3):
        assert lib.tmvs_status_string(code)
    assert lib.tmvs_status_string(0) != lib.tmvs_status_string(-2)


def test_bn_fold_host(lib):
    """tmvs_bn_fold is host code: alpha = gamma/sqrt(var+eps) (reference op order), shift = beta - mean*alpha."""
    g = np.random.default_rng(0)
    gamma, beta, mean = (g.standard_normal(16).astype(np.float32) for _ in range(3))
    var = g.random(16).astype(np.float32) + 0.1
    alpha = np.empty(16, np.float32)
    shift = np.empty(16, np.float32)
    p = lambda a: a.ctypes.data
    assert lib.tmvs_bn_fold(p(gamma), p(beta), p(mean), p(var), 16, 1e-5, p(alpha), p(shift)) == 0
    ea = (np.float32(1) / np.sqrt(var + np.float32(1e-5))) * gamma
    np.testing.assert_array_equal(alpha, ea)
    np.testing.assert_allclose(shift, beta - mean * ea, rtol=0, atol=1e-6)


def test_argument_validation_without_gpu(lib):
    """Null pointers / unsupported shapes are rejected before any launch."""
    assert lib.tmvs_warp_corr(None, None, None, None, None, 0, 0, 4, None, 1, 4, 32, 48, 8, 8, 0,
                              None, None, None, None) == -1
    assert lib.tmvs_softmax_wta(None, None, 1, 48, 8, 8, 425.0, 935.0, None, None, None, None, None) == -1
    assert lib.tmvs_costregnet_workspace(1, 48, 216, 288, 8) > 0
    assert lib.tmvs_depth_stage_workspace(48, 216, 288, 8) > lib.tmvs_costregnet_workspace(1, 48, 216, 288, 8)
    # the grouped K/V: a view subset keeps the tiling of the larger launch, so its slab is the subset's share
    L = 216 * 288
    assert lib.tmvs_fmt_kv_grouped_workspace(5, 5, L) == lib.tmvs_fmt_kv_workspace(5, L)
    assert 5 * lib.tmvs_fmt_kv_grouped_workspace(1, 5, L) == lib.tmvs_fmt_kv_workspace(5, L)
    assert lib.tmvs_fmt_kv_grouped_workspace(1, 1, L) == lib.tmvs_fmt_kv_workspace(1, L)
    assert lib.tmvs_fmt_kv_grouped_workspace(0, 5, L) == 0
    assert lib.tmvs_fmt_kv_grouped(None, 1, 5, L, None, None, 0, None, None) == -1
    # the split FMT needs both K/V slabs; NULL side stream falls back to (and validates like) tmvs_fmt_forward
    assert lib.tmvs_fmt_forward_split_workspace(5, L) > lib.tmvs_fmt_forward_workspace(5, L)
    assert lib.tmvs_fmt_forward_split_workspace(1, L) == lib.tmvs_fmt_forward_workspace(1, L)
    assert lib.tmvs_fmt_forward_split(None, 0, None, 0, 0, 5, 216, 288, None, None, 0, None, None, None) == -1


def test_forward_refuses_cpu_tensors():
    from transmvsnet_amd import TransMVSNet, synthetic
    m = TransMVSNet(ndepths=[8, 8, 8]).eval()
    feats = synthetic.synthetic_features(3, 64, 80)
    proj = synthetic.synthetic_cameras(3, 64, 80)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m.forward_features(feats, proj, synthetic.synthetic_depth_values(1), (64, 80))


def test_deform_conv2d_pack_host(lib):
    """tmvs_deform_conv2d_pack (HOST): A fragments [tap][mtile][half][lane][e], k-step s = 4*half + e feeds
    channel 16*half + 4*(lane/16) + e (the kernel's B lanes hold channels 4j..4j+3 and 16+4j..16+4j+3)."""
    import numpy as np
    import torch
    from transmvsnet_amd import ops
    for co in (8, 16, 32):
        w = torch.randn(co, 32, 3, 3)
        pk = ops.deform_conv2d_pack(w).numpy()
        mt_n = (co + 15) // 16
        assert pk.size == 9 * 8 * mt_n * 64
        wn = w.numpy()
        for k in (0, 4, 8):
            for s in (0, 3, 7):
                for mt in range(mt_n):
                    for lane in (0, 5, 17, 63):
                        h, e = s // 4, s % 4
                        c_o, c_i = 16 * mt + lane % 16, 16 * h + 4 * (lane // 16) + e
                        want = wn[c_o, c_i, k // 3, k % 3] if c_o < co else 0.0
                        assert pk[((((k * mt_n + mt) * 2 + h) * 64) + lane) * 4 + e] == want


def test_conv2d_pack_host(lib):
    """tmvs_conv2d_pack (HOST): [k-block][mtile][lane][e]; lane group j of k-block b owns the (tap, chunk) pair
    idx = 4b + j, element e = channel 4*chunk + e; zero padding past cin / cout / the last pair."""
    import numpy as np
    import torch
    from transmvsnet_amd import ops
    for (co, ci, k) in ((8, 3, 3), (16, 8, 5), (32, 32, 1), (32, 16, 3)):
        w = torch.randn(co, ci, k, k)
        pk = ops.conv2d_pack(w).numpy()
        cip = max(ci, 4)
        g = cip // 4
        nidx = k * k * g
        nb, mt = (nidx + 3) // 4, (co + 15) // 16
        assert pk.size == nb * mt * 64 * 4
        wn = w.numpy()
        for b in range(nb):
            for m in range(mt):
                for lane in (0, 7, 21, 63):
                    for e in range(4):
                        idx, c_o = 4 * b + lane // 16, 16 * m + lane % 16
                        want = 0.0
                        if idx < nidx and c_o < co:
                            tap, c = idx // g, 4 * (idx % g) + e
                            if c < ci:
                                want = wn[c_o, c, tap // k, tap % k]
                        assert pk[((b * mt + m) * 64 + lane) * 4 + e] == want


def test_host_rot_order_matches_torch_matmul():
    """ops.host_rot_order names the rounding this host's torch.matmul gives rot·(x, y, 1) (the
    reference's homo_warping grid, models/module.py:303); emulate it and compare bit for bit."""
    import numpy as np
    import torch
    from transmvsnet_amd import ops
    h, w = 216, 288
    order = ops.host_rot_order(h * w)
    assert order in ("fma", "plain")
    assert ops.warp_flags("auto", h * w) == (_lib.WARP_ROT_PLAIN if order == "plain" else 0)
    assert ops.warp_flags("fma", h * w) == 0 and ops.warp_flags("plain", h * w) == _lib.WARP_ROT_PLAIN
    rot = np.float32([[0.99, -0.02, -3.1], [0.015, 1.01, 2.7], [1.2e-5, -3e-6, 1.0]])
    y, x = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32), indexing="ij")
    x, y = x.reshape(-1), y.reshape(-1)
    got = torch.matmul(torch.from_numpy(rot)[None], torch.from_numpy(np.stack([x, y, np.ones_like(x)]))[None])[0]
    r0, r1, r2 = rot[:, 0:1], rot[:, 1:2], rot[:, 2:3]
    if order == "fma":
        emu = (r1.astype(np.float64) * y + (r0 * x)).astype(np.float32) + r2
    else:
        emu = (r0 * x + r1 * y) + r2
    assert (emu == got.numpy()).mean() == 1.0


def test_training_host_logic():
    """Training-path host logic (no GPU): the FMT weight block _FMTTrain packs from the 16 layer
    parameters is exactly EncoderLayer.packed() (the tmvs_fmt_* layout, include/transmvs.h
    TMVS_ENC_*); fmt_params walks the 8 layers in _ENC_PARAMS order; every training entry point
    refuses CPU tensors instead of falling back."""
    import torch
    from transmvsnet_amd import TransMVSNet
    from transmvsnet_amd.train import (_ENC_PARAMS, _pack_enc, costregnet_train, fmt_params, fmt_train,
                                       pathway_train, warp_corr_views)
    m = TransMVSNet()
    layers = m.FMT_with_pathway.FMT.layers
    ps = fmt_params(m)
    assert len(ps) == 8 * len(_ENC_PARAMS) == 128
    for i, layer in enumerate(layers):
        named = dict(layer.named_parameters())
        assert all(ps[16 * i + j] is named[n] for j, n in enumerate(_ENC_PARAMS))
        assert torch.equal(_pack_enc(ps[16 * i:16 * i + 16]), layer.packed())
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        fmt_train(m, torch.zeros(3, 32, 8, 10))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        warp_corr_views(torch.zeros(8, 10, 32), torch.zeros(2, 8, 10, 32), torch.zeros(4, 8, 10), None)
    with pytest.raises(RuntimeError):
        costregnet_train(m.cost_regularization[0], torch.zeros(1, 8, 16, 16))
    with pytest.raises(RuntimeError):
        pathway_train(m, torch.zeros(3, 8, 10, 32), torch.zeros(3, 16, 16, 20), torch.zeros(3, 8, 32, 40))


def test_every_launching_op_is_device_guarded():
    """Every public op in ops.py that launches on the current stream (_stream()) runs under the
    device guard of its first GPU tensor argument (costregnet_wta was missing)."""
    import inspect

    from transmvsnet_amd import ops
    missing = []
    for name, fn in vars(ops).items():
        if name.startswith("_") or not inspect.isfunction(fn) or fn.__module__ != ops.__name__:
            continue
        src = inspect.getsource(inspect.unwrap(fn))
        if "_stream()" in src and not getattr(fn, "device_guarded", False):
            missing.append(name)
    assert not missing, missing


def test_training_device_packs_equal_host_packs():
    """featurenet_train packs weights on the device (no host sync per step) with index gathers that
    must reproduce the host packers tmvs_conv2d_pack / tmvs_deform_conv2d_pack bit for bit."""
    import torch

    from transmvsnet_amd import ops
    from transmvsnet_amd.featurenet_train import device_pack
    g = torch.Generator().manual_seed(0)
    for co, ci, k in ((8, 3, 3), (8, 8, 3), (16, 8, 5), (16, 16, 3), (32, 16, 5), (32, 32, 3), (32, 32, 1)):
        w = torch.randn(co, ci, k, k, generator=g)
        assert torch.equal(ops.conv2d_pack(w), device_pack("conv2d", w)), (co, ci, k)
    for co in (8, 16, 27, 32):
        w = torch.randn(co, 32, 3, 3, generator=g)
        assert torch.equal(ops.deform_conv2d_pack(w), device_pack("dcn", w)), co
