"""Which side of an fp32 near tie exact arithmetic is on, and how far the reference moves itself (CPU only).

For one full-size configuration (bench inputs: stacked_features SEED, synthetic_cameras seed 1, key-seeded
weights with logit sharpening) and a list of (stage, y, x) pixels:
  * the fp32 oracle cascade (= the reference's arithmetic), at THREADS torch threads and at ALT_THREADS
    (MKL / oneDNN blocking changes with the thread count): per stage, the pixels where the two reference
    runs disagree and the cascaded mean |depth difference| between them -- the reference's own spread;
  * the stage in float64 (FMT + pathway features, cost volume with the stage-1 view weights, CostRegNet),
    built on the fp32 reference's previous-stage depth (the same hypotheses as the fp32 runs): argmax and
    top-2 log-probability margin at each listed pixel, next to the fp32 reference's.

    python scripts/diag/exact_pick.py NVIEWS H W SEED STAGE:Y:X [STAGE:Y:X ...]
Env: THREADS (default 8), ALT_THREADS (default 1; 0 = skip the self-consistency run).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import parity  # noqa: E402
from oracle import transmvs_ref as oracle  # noqa: E402
from transmvsnet_amd import TransMVSNet, synthetic  # noqa: E402


def log(*a):
    print(*a, flush=True)


def top2(lg_col):
    x = lg_col.double()
    lp = x - torch.logsumexp(x, 0)
    s = torch.sort(lp, descending=True)
    return int(s.indices[0]), int(s.indices[1]), float(s.values[0] - s.values[1])


def main():
    n, H, W, seed = (int(a) for a in sys.argv[1:5])
    pix = [tuple(int(v) for v in a.split(":")) for a in sys.argv[5:]]
    nt, alt = int(os.environ.get("THREADS", "8")), int(os.environ.get("ALT_THREADS", "0"))
    sd = synthetic.synthetic_state_dict(synthetic.state_dict_shapes(TransMVSNet()), seed=0, sharpen=100.0)
    feats_cpu = synthetic.stacked_features(n, H, W, seed=seed)
    proj = synthetic.synthetic_cameras(n, H, W, seed=1)
    dv = synthetic.synthetic_depth_values(1)
    views = [{k: v[:, i] for k, v in feats_cpu.items()} for i in range(n)]
    with torch.no_grad():
        torch.set_num_threads(nt)
        ref = oracle.forward_from_features(sd, views, proj, dv, (H, W))
        log(f"fp32 reference at {nt} threads done")
        if alt > 0:
            torch.set_num_threads(alt)
            ref2 = oracle.forward_from_features(sd, views, proj, dv, (H, W))
            torch.set_num_threads(nt)
            rep = parity.cascade_report(ref2, ref)
            for s in (1, 2, 3):
                r = rep[f"cascade_stage{s}"]
                log(f"reference {alt} vs {nt} threads, stage {s}: mean |d| {r['mean_abs_mm']:.3g} mm, {r['differing']} "
                    f"differing ({r['near_tie_flips']} near ties, {r['cascade_explained']} cascaded, {r['other_flips']} "
                    f"other), pixels {r['differing_pixels'][:8]}")
        sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
        views64 = [{k: v.double() for k, v in f.items()} for f in views]
        f64 = oracle.fmt_with_pathway(sd64, views64)
        log("float64 features done")
        # float64 stage-1 view weights (stage-1 hypotheses are the depth_values planes on both sides)
        hyp1 = oracle.stage_hypotheses(None, dv, 0, (H, W)).double()
        _, vw64 = oracle.build_cost_volume(sd64, [f["stage1"] for f in f64], proj["stage1"].double(), hyp1)
        for stage in sorted({p[0] for p in pix}):
            s = stage - 1
            name = f"stage{stage}"
            prev = None if s == 0 else parity.raw_depth(ref[f"stage{s}"])
            hyp = oracle.stage_hypotheses(prev, dv, s, (H, W))
            assert torch.equal(hyp, ref[name]["depth_values"])
            vw_up = None
            if s > 0:
                vw_up = vw64
                for _ in range(s):
                    vw_up = F.interpolate(vw_up, scale_factor=2, mode="nearest")
            sim, _ = oracle.build_cost_volume(sd64, [f[name] for f in f64], proj[name].double(), hyp.double(), vw_up)
            lg = oracle.cost_reg_net(sd64, f"cost_regularization.{s}.", sim).reshape(1, -1, *hyp.shape[-2:])
            lp32 = torch.log(ref[name]["prob_volume"].double())
            for st, y, x in pix:
                if st != stage:
                    continue
                a64, b64, m64 = top2(lg[0, :, y, x])
                s32 = torch.sort(lp32[0, :, y, x], descending=True)
                log(f"{name} ({y},{x}): fp32 reference picks {int(s32.indices[0])} over {int(s32.indices[1])} by "
                    f"{float(s32.values[0] - s32.values[1]):.3g}; float64 picks {a64} over {b64} by {m64:.3g}")


if __name__ == "__main__":
    main()
