"""packing.gather_packs (CPU): one cat + index gather equals applying each re-layout to its tensor, for
the CostRegNet training packings (forward, data gradient incl. flipped / prob_kernel layouts, weight
gradient unpacking) and the FMT's multi-tensor layer block."""
import torch

from transmvsnet_amd import train
from transmvsnet_amd.packing import gather_packs


def test_costregnet_packs_equal_direct_relayouts():
    g = torch.Generator().manual_seed(0)
    ws = []
    for name, stride, transposed, _ in train._LAYERS:
        ci, co = {"conv0": (1, 8), "conv1": (8, 16), "conv2": (16, 16), "conv3": (16, 32), "conv4": (32, 32),
                  "conv5": (32, 64), "conv6": (64, 64), "conv7": (64, 32), "conv9": (32, 16), "conv11": (16, 8)}[name]
        ws.append(torch.randn((ci, co, 3, 3, 3) if transposed else (co, ci, 3, 3, 3), generator=g))
    ws.append(torch.randn(1, 8, 3, 3, 3, generator=g))
    geo = [(i, *train._layer_channels(ws[i], tr), st, tr) for i, (_, st, tr, _) in enumerate(train._LAYERS)]
    geo.append((len(train._LAYERS), 8, 1, 1, False))
    fns = [train._fwd_pack_fn(ci, co, st, tr) for _, ci, co, st, tr in geo] + \
          [train._dgrad_pack_fn(ci, co, st, tr) for _, ci, co, st, tr in geo]
    idx = [i for i, *_ in geo] * 2
    got = gather_packs(ws, list(zip(idx, fns)), "test_costregnet")
    for (i, fn), t in zip(zip(idx, fns), got):
        assert torch.equal(t, fn(ws[i]).contiguous())
    # second call: the cached index map, new values
    ws2 = [w * 3 + 1 for w in ws]
    got2 = gather_packs(ws2, list(zip(idx, fns)), "test_costregnet")
    for (i, fn), t in zip(zip(idx, fns), got2):
        assert torch.equal(t, fn(ws2[i]).contiguous())
    shapes = [w.shape for w in ws]
    dws = [torch.randn(27, s[0], s[1], generator=g) for s in shapes]
    unp = gather_packs(dws, [(i, (lambda t, s=s_: train._unpack_wgrad(t, s))) for i, s_ in enumerate(shapes)], "test_unp")
    for d, s, u in zip(dws, shapes, unp):
        assert torch.equal(u, train._unpack_wgrad(d, s))


def test_multi_tensor_spec_and_zero_padding():
    a, b = torch.randn(3, 4), torch.randn(2, 5)
    fn = lambda x, y: torch.cat([x.t().reshape(-1), torch.zeros(3), y.flip(1).reshape(-1)])  # noqa: E731
    (out,) = gather_packs([a, b], [((0, 1), fn)], "test_multi")
    assert torch.equal(out, fn(a, b))


def test_fmt_layer_blocks():
    g = torch.Generator().manual_seed(1)
    from transmvsnet_amd import TransMVSNet
    params = [p.detach() + torch.randn(p.shape, generator=g) for p in train.fmt_params(TransMVSNet())]
    enc = gather_packs(params, [(tuple(range(16 * i, 16 * i + 16)), lambda *p: train._pack_enc(p)) for i in range(8)],
                       "test_fmt")
    for i in range(8):
        assert torch.equal(enc[i], train._pack_enc(params[16 * i:16 * i + 16]))


def test_offset_conv_dgrad_pack_one_gather():
    """featurenet_train.offset_dgrad_pack (one gather from conv_offset_mask.weight) equals the DCN
    backward's previous build of the same pack: the weight zero-padded to 32 output rows, flipped and
    transposed (dgrad_same's weight), then device_pack('dcn', .)."""
    from transmvsnet_amd import featurenet_train as ft
    g = torch.Generator().manual_seed(1)
    for _ in range(2):
        w = torch.randn(27, 32, 3, 3, generator=g)
        wp = torch.zeros(32, 32, 3, 3)
        wp[:27] = w
        assert torch.equal(ft.offset_dgrad_pack(w), ft.device_pack("dcn", ft._flip_t(wp)))
