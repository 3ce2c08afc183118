"""B > 1 with the samples on concurrent streams, captured as one HIP graph (needs an MI355X; -m gpu).

models/TransMVSNet.py:141-226 computes each sample of a batch independently (stages 2/3 take the
hypothesis interval from depth_values[0], :146-148). TransMVSNet.forward_features runs sample i > 0 on
its own stream (forked from and joined back into the caller's stream; each sample stream forks its own
FMT-pathway side stream). Round 5 disabled that fork inside a graph capture after a segfault seen only
under `rocprofv3 --kernel-trace` (gpurun_out/r16c/ab.txt); this test captures the fork at the bench's
full size, B = 2, and requires replay == eager == the sequential form, bit for bit.
"""
import pytest
import torch

from transmvsnet_amd import TransMVSNet, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"
KEYS = ("depth", "photo_confidence", "prob_volume", "depth_values")


def test_batch2_full_size_capture_equals_eager():
    H, W, N = 864, 1152, 5
    m = TransMVSNet().eval()
    m.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=0, sharpen=100.0))
    m = m.to(DEV)
    fs = [synthetic.stacked_features(N, H, W, seed=2 + 3 * b) for b in range(2)]
    feats = {k: torch.cat([f[k] for f in fs], 0).to(DEV).contiguous() for k in fs[0]}
    cams = [synthetic.synthetic_cameras(N, H, W, seed=1 + b) for b in range(2)]
    proj = {k: torch.cat([c[k] for c in cams], 0) for k in cams[0]}
    dv = torch.cat([synthetic.synthetic_depth_values(1), synthetic.synthetic_depth_values(1) + 2.0], 0).to(DEV)
    with torch.no_grad():
        m.batch_streams = False
        try:
            seq = m.forward_features(feats, proj, dv, (H, W))
        finally:
            m.batch_streams = True
        con = m.forward_features(feats, proj, dv, (H, W))
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_out = m.forward_features(feats, proj, dv, (H, W))
        torch.cuda.synchronize()
        for _ in range(3):
            graph.replay()
        torch.cuda.synchronize()
    for s in (1, 2, 3):
        for k in KEYS:
            a = seq[f"stage{s}"][k]
            assert torch.equal(a, con[f"stage{s}"][k]), (s, k, "concurrent eager")
            assert torch.equal(a, g_out[f"stage{s}"][k]), (s, k, "graph replay")


# The B = 1 step's stream layouts -- one stream (no overlap, one-stream FMT), the FMT's reference chain on a
# side stream (tmvs_fmt_forward_split), the pathway forked after stage 1's cost volume or right after the FMT,
# the FMT and the pathway on one side stream -- give the same bits, eager and as a replayed graph.
@pytest.mark.parametrize("layout", ["split", "split_fmtfork", "split_fmtfork_oneside", "split_fmtfork_join2"])
def test_stream_layouts_bitwise(layout):
    H, W, N = 512, 640, 5
    m = TransMVSNet().eval()
    m.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=0, sharpen=100.0))
    m = m.to(DEV)
    feats = {k: v.to(DEV).contiguous() for k, v in synthetic.stacked_features(N, H, W, seed=4).items()}
    proj = synthetic.synthetic_cameras(N, H, W, seed=3)
    dv = synthetic.synthetic_depth_values(1).to(DEV)
    with torch.no_grad():
        m.overlap_pathway, m.split_fmt = False, False
        ref = m.forward_features(feats, proj, dv, (H, W))
        m.overlap_pathway, m.split_fmt = True, True
        m.pathway_fork = "fmt" if "fmtfork" in layout else "warp"
        m.one_side_stream = "oneside" in layout
        m.pathway_join2 = "join2" in layout
        eager = m.forward_features(feats, proj, dv, (H, W))
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            g_out = m.forward_features(feats, proj, dv, (H, W))
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()
    for s in (1, 2, 3):
        for k in KEYS:
            a = ref[f"stage{s}"][k]
            assert torch.equal(a, eager[f"stage{s}"][k]), (layout, s, k, "eager")
            assert torch.equal(a, g_out[f"stage{s}"][k]), (layout, s, k, "graph replay")
