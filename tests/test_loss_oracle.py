"""Loss oracle (oracle/loss_ref.py) against the reference's own outputs (tests/golden/loss.npz,
made by tests/golden/make_golden_loss.py from models/module.py). CPU only."""
import os

import numpy as np
import pytest
import torch

from oracle import loss_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden", "loss.npz")
STAGES = ("stage1", "stage2", "stage3")


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD) as z:
        return {k: z[k] for k in z.files}


def _case(gold, p):
    t = lambda k: torch.from_numpy(gold[f"{p}_{k}"])  # noqa: E731
    logits = {s: t(f"{s}_logits") for s in STAGES}
    dvs = {s: t(f"{s}_dv") for s in STAGES}
    gts = {s: t(f"{s}_gt") for s in STAGES}
    masks = {s: t(f"{s}_mask") for s in STAGES}
    return logits, dvs, gts, masks


def test_trans_mvsnet_loss_and_grads_bit_exact(gold):
    logits, dvs, gts, masks = _case(gold, "t")
    (total, depth_loss, total_entropy, depth_entropy), grads = loss_ref.loss_and_logit_grads(
        logits, dvs, gts, masks, dlossw=[0.5, 1.0, 2.0])
    assert total.item() == gold["t_total"]
    assert depth_loss.item() == gold["t_depth_loss"]
    assert total_entropy.item() == gold["t_total_entropy"]
    assert np.array_equal(depth_entropy.numpy(), gold["t_depth_entropy"])
    for s in STAGES:
        assert np.array_equal(grads[s].numpy(), gold[f"t_{s}_grad"]), s


def test_entropy_loss_prob_map_bit_exact(gold):
    logits, dvs, gts, masks = _case(gold, "t")
    p = torch.softmax(logits["stage2"], dim=1)
    loss, wta, conf = loss_ref.entropy_loss(p, gts["stage2"], masks["stage2"] > 0.5, dvs["stage2"],
                                            return_prob_map=True)
    assert loss.item() == gold["e_loss"]
    assert np.array_equal(wta.numpy(), gold["e_wta"])
    assert np.array_equal(conf.numpy(), gold["e_conf"])


def test_focal_loss_bld_bit_exact(gold):
    logits, dvs, gts, masks = _case(gold, "f")
    depth3 = torch.from_numpy(gold["f_depth3"])
    interval = torch.from_numpy(gold["f_interval"])

    def fn(inputs):
        inputs["stage3"]["depth"] = depth3
        return loss_ref.focal_loss_bld(inputs, gts, masks, interval)

    res, grads = loss_ref.loss_and_logit_grads(logits, dvs, gts, masks, loss_fn=fn)
    for name, v in zip(("total", "depth_loss", "epe", "less1", "less3"), res):
        assert v.item() == gold[f"f_{name}"], name
    for s in STAGES:
        assert np.array_equal(grads[s].numpy(), gold[f"f_{s}_grad"]), s
