"""The cost-volume kernels (tmvs_warp_corr) on COHERENT stage-2/3 hypotheses next to the bench's own.

The bench's features are random, so its stage-1/2 winner-take-all depth -- from which the stage-2/3
hypotheses are built (models/TransMVSNet.py:174-190) -- is spatially incoherent, and the bilinear taps of
neighbouring pixels land in unrelated source neighbourhoods (L1 misses, 29 address-unit
cycles per load instruction at stage 3). Real scenes give smooth depth. Here the same stage features,
cameras, view weights and kernels run with the hypotheses built by tmvs_stage_hypotheses from a smooth
previous-stage depth -- a slanted plane through the DTU depth range, 600 + 150 x/W + 100 y/H mm -- against
the bench's (from the GPU's own stage-1/2 WTA depth). Per stage: HIP-event median of REPS launches, the
bilinear tap bytes 16 C D P V over that time against the address unit's 39.3 TB/s, and the algorithmic HBM
bytes over it against 8 TB/s.

    python scripts/diag/warp_coherent.py [REPS] [--json OUT]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from transmvsnet_amd import TransMVSNet, ops, synthetic  # noqa: E402
from transmvsnet_amd.model import STAGE_SCALES  # noqa: E402

TA_PEAK = 64 * 256 * 2.4e9  # B/s: the measured 64 B/clk/CU address-unit rate
HBM_PEAK = 8.0e12


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else 20
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    dev = torch.device("cuda", 0)
    H, W, N = bench.H, bench.W, bench.NVIEWS
    m = TransMVSNet().eval()
    m.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(m), seed=0, sharpen=100.0))
    m = m.to(dev)
    feats_cpu, proj, dv = bench.make_inputs(dev)
    feats = {k: v.to(dev) for k, v in feats_cpu.items()}
    dv = dv.to(dev)
    with torch.no_grad():
        out, vw = m.forward_features(feats, proj, dv, (H, W), return_view_weights=True)
        prep = m._prepared(dev)
        s1, s2, s3 = feats["stage1"][0], feats["stage2"][0], feats["stage3"][0]
        n, _, h1, w1 = s1.shape
        st1 = m._fmt(s1, prep).view(n, h1, w1, 32)
        st2 = ops.fmt_pathway(st1, s2, prep["red1"], prep["sm1"])
        st3 = ops.fmt_pathway(st2, s3, prep["red2"], prep["sm2"])
        fs = (st1, st2, st3)
    rows = {k: ops.proj_rows(proj[k]) for k in ("stage1", "stage2", "stage3")}
    res = {"workload": f"DTU {H}x{W}, N={N}, 48/32/8: the bench's stage features, cameras and view weights",
           "coherent": "stage-2/3 hypotheses from the plane depth 600 + 150 x/W + 100 y/H mm (tmvs_stage_hypotheses)",
           "bench": "stage-2/3 hypotheses from the GPU's own stage-1/2 WTA depth on the random-feature bench input",
           "reps": reps, "stages": {}}
    for s in (1, 2):
        name = f"stage{s + 1}"
        hp, wp = H // STAGE_SCALES[s - 1], W // STAGE_SCALES[s - 1]
        yy, xx = torch.meshgrid(torch.arange(hp, dtype=torch.float32), torch.arange(wp, dtype=torch.float32), indexing="ij")
        plane = (600.0 + 150.0 * xx / wp + 100.0 * yy / hp)[None].to(dev).contiguous()
        hyps = {"bench": out[name]["depth_values"].contiguous(),
                "coherent": ops.stage_hypotheses(dv[0:1], plane, m.ndepths[s], m.depth_interals_ratio[s], (H, W),
                                                 STAGE_SCALES[s])}
        f = fs[s]
        ref, src = f[0:1], f[1:].unsqueeze(0)
        _, h, w, c = f.shape
        d = m.ndepths[s]
        v = N - 1
        p = h * w
        tap_bytes = 16 * c * d * p * v
        alg_bytes = 4 * p * (c * (1 + v) + 2 * d + v)
        row = {}
        for kind, hyp in hyps.items():
            for _ in range(3):
                ops.warp_corr(ref, src, rows[name], hyp, view_w_in=vw, vw_shift=s)
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.warp_corr(ref, src, rows[name], hyp, view_w_in=vw, vw_shift=s)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            us = float(np.median(ts))
            row[kind] = {"us": round(us, 2), "gather_frac_of_ta": round(tap_bytes / (us * 1e-6) / TA_PEAK, 4),
                         "hbm_frac": round(alg_bytes / (us * 1e-6) / HBM_PEAK, 4),
                         "hyp_spread_mm": round(float((hyp[:, 1:] - hyp[:, :-1]).abs().mean()), 4)}
        res["stages"][name] = row
        print(name, json.dumps(row), flush=True)
    if out_json:
        os.makedirs(os.path.dirname(out_json), exist_ok=True)
        with open(out_json, "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()
