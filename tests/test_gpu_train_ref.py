"""The HIP training path against the REFERENCE's own training step (tests/golden/train_c1.npz, made by
tests/golden/make_golden_train.py from /root/reference: finetune.py:144-168's train_sample body at C1
size, 128x160, N=3, 8/8/8, key-seeded weights, prob.weight x10). Needs an MI355X (-m gpu).

  * from features (case "f"): fmt_train -> pathway_train -> depth_stages_forward_train ->
    transmvsnet_amd.loss.focal_loss_bld(...)[0].backward(): the loss terms, WTA depths, prob volumes,
    the gradient of every FMT / pathway / PixelwiseNet / CostRegNet parameter and of the stage
    features, the BatchNorm running statistics;
  * from images (case "i"), the reference's train_sample body unchanged on the drop-in model:
        model.train(); optimizer.zero_grad(); outputs = model(imgs, proj_matrix, depth_values)
        loss, depth_loss, epe, less1, less3 = focal_loss_bld(outputs, depth_gt_ms, mask_ms, interval,
                                                             dlossw=[1.0, 1.0, 1.0])
        loss.backward(); optimizer.step()
    with focal_loss_bld both the HIP loss (transmvsnet_amd.loss) and the reference's torch-op loss
    (restated in oracle/loss_ref.py, the code a reference user already calls), which backpropagates
    through prob_volume (the HIP softmax backward). All 318 parameter gradients incl. FeatureNet +
    DCN (models/module.py:343-422, models/dcn.py:66-80), and the running statistics.

Bar: the reference's fp32 numbers are themselves rounded; every gradient is compared with a float64
evaluation of the same step (the oracle, pinned bit-exact to these fixtures by
tests/test_train_oracle.py) and must be within max(1e-4, 2x the fp32 spread) of its max magnitude,
the fp32 spread being the worst distance from fp64 over the fixture's own fp32 run and 4 fp32 oracle
runs whose inputs are jittered by ~1 ulp (some gradients are ill-conditioned: at C1 a 2e-7 input
jitter moves the reference's stage-3 conv5 gradient between 1e-3 and 4e-2 of its magnitude, a ReLU /
argmax flip away; scripts/diag/train_cond.py, profiles/r09c/); loss terms within 1e-5
relative, prob volumes within max(1e-4, 3x the fp32 reference's distance from fp64), WTA depths
identical outside the 1e-4 near-tie margin, running statistics within 1e-5.
"""
import numpy as np
import pytest
import torch

from tests._util import golden_rot, golden_state_dict
from tests.test_train_oracle import GOLD, H, ND, N, STAGES, TRAIN_SHARPEN, train_step_oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD) as z:
        return {k: z[k] for k in z.files}


ENSEMBLE = 4  # perturbed fp32 oracle runs per case


@pytest.fixture(scope="module")
def exact():
    """Per case: float64 evaluations (the CPU oracle) and, per gradient, the worst relative distance
    from them over the fixture's fp32 run and ENSEMBLE fp32 oracle runs with ~1-ulp input jitter."""
    with np.load(GOLD) as z:
        g = {k: z[k] for k in z.files}
    torch.set_num_threads(min(16, torch.get_num_threads()))
    out = {}
    for case in ("f", "i"):
        res, o, sd, leaves = train_step_oracle(g, case, dtype=torch.float64)
        grads = {k: v.grad.detach().numpy() for k, v in sd.items() if v.requires_grad and v.grad is not None}
        fg = {} if leaves is None else {f"{v}_{k}": t.grad.numpy() for v, f in enumerate(leaves) for k, t in f.items()}
        prob = {s: o[f"stage{s}"]["prob_volume"].detach().numpy() for s in (1, 2, 3)}
        spread = {n: _rel(g[f"{case}_grad.{n}"], grads[n]) for n in grads}
        for e in range(ENSEMBLE):
            sd_e = train_step_oracle(g, case, perturb_seed=1000 + e)[2]
            for n in grads:
                spread[n] = max(spread[n], _rel(sd_e[n].grad.detach().numpy(), grads[n]))
        out[case] = (grads, fg, prob, spread)
    return out


def _model():
    from transmvsnet_amd import TransMVSNet
    m = TransMVSNet(ndepths=list(ND))
    m.load_state_dict(golden_state_dict(sharpen=TRAIN_SHARPEN), strict=True)
    return m.to(DEV)


def _targets(gold):
    gt = {s: torch.from_numpy(gold[f"gt_{s}"]).to(DEV) for s in STAGES}
    mask = {s: torch.from_numpy(gold[f"mask_{s}"]).to(DEV) for s in STAGES}
    return gt, mask


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max()) / max(float(np.abs(b).max()), 1e-30)


def _judge(gold, ex, case, got):
    """got: {name: gradient (numpy)} -> report; asserts the module docstring's bar.

    A gradient that is zero in exact arithmetic (a bias feeding a train-mode BatchNorm: the batch
    mean removes it, e.g. feature.out*.{1,4}.bias) has no relative scale: it is judged in absolute
    terms, within 3x the fp32 reference's own absolute noise, and kept out of the shared bar."""
    exact_grads, spread = ex[0], ex[3]
    pfx = f"{case}_grad."
    names = sorted(k[len(pfx):] for k in gold if k.startswith(pfx))
    missing = [n for n in names if n not in got]
    assert not missing, f"no gradient for {missing[:8]} ({len(missing)} of {len(names)})"
    scale = float(np.median([np.abs(exact_grads[n]).max() for n in names]))
    degenerate = {n for n in names if float(np.abs(exact_grads[n]).max()) < 1e-7 * scale}
    rows = []
    for n in names:
        if n in degenerate:
            e = float(np.abs(np.asarray(got[n], np.float64) - exact_grads[n]).max())
            f = float(np.abs(gold[pfx + n].astype(np.float64) - exact_grads[n]).max())
            assert e <= max(3.0 * f, 1e-7 * scale), (n, "exactly-zero gradient", e, f)
            continue
        e = _rel(got[n], exact_grads[n])
        bar = max(1e-4, 2.0 * spread[n])
        rows.append((e / bar, n, e, spread[n]))
    rows.sort(reverse=True)
    print(f"{case}: {len(rows)} gradients (+{len(degenerate)} exactly zero in fp64); worst errors vs fp64 "
          f"(ratio to bar, name, gpu, fp32 spread):", [(f"{r:.2f}", n, f"{e:.1e}", f"{f:.1e}") for r, n, e, f in
                                                     rows[:8]])
    bad = [(n, e, f) for r, n, e, f in rows if r > 1.0]
    assert not bad, bad[:10]


def _check_outputs(gold, case, outputs, loss_terms, exact_prob):
    for name, v in zip(("loss", "depth_loss", "epe", "less1", "less3"), loss_terms):
        ref = float(gold[f"{case}_{name}"])
        assert abs(float(v) - ref) <= 1e-5 * max(abs(ref), 1.0), (name, float(v), ref)
    rep = {}
    for s in (1, 2, 3):
        o = outputs[f"stage{s}"]
        np.testing.assert_array_equal(o["depth_values"].detach().cpu().numpy(), gold[f"{case}_stage{s}_hyp"])
        ref = gold[f"{case}_stage{s}_prob"].astype(np.float64)
        # WTA depth identical except where the reference's top-2 log-prob margin is a near tie
        srt = np.sort(ref, axis=1)
        near = (np.log(np.maximum(srt[:, -1], 1e-30)) - np.log(np.maximum(srt[:, -2], 1e-30))) < 1e-4
        diff = o["depth"].detach().cpu().numpy() != gold[f"{case}_stage{s}_depth"]
        assert not (diff & ~near).any(), (s, int(diff.sum()), int((diff & ~near).sum()))
        # prob volumes: against float64, within 3x the fp32 reference's own distance (or 1e-4)
        ex = exact_prob[s]
        e_gpu = float(np.abs(o["prob_volume"].detach().cpu().numpy() - ex).max())
        e_ref = float(np.abs(ref - ex).max())
        rep[s] = (e_gpu, e_ref)
        assert e_gpu <= max(1e-4, 3.0 * e_ref), (s, e_gpu, e_ref)
    print(case, "prob vs fp64 per stage (gpu, fp32 reference):", rep)


def _check_buffers(gold, case, model):
    bufs = dict(model.named_buffers())
    worst = 0.0
    for k in gold:
        if k.startswith(f"{case}_buf."):
            n = k[len(case) + 5:]
            if n.endswith("num_batches_tracked"):
                assert int(bufs[n]) == int(gold[k]), n
            else:
                worst = max(worst, float(np.abs(bufs[n].cpu().numpy() - gold[k]).max()))
    assert worst < 1e-5, worst


def test_train_step_from_features_vs_reference(gold, exact):
    from transmvsnet_amd import loss as hip_loss
    from transmvsnet_amd import synthetic
    from transmvsnet_amd.train import depth_stages_forward_train, fmt_train, pathway_train
    model = _model()
    model.train()
    feats = synthetic.synthetic_features(N, H, H * 5 // 4, seed=2)
    leaves = {k: torch.cat([f[k] for f in feats], 0).to(DEV).requires_grad_() for k in STAGES}
    proj = synthetic.synthetic_cameras(N, H, H * 5 // 4, seed=1)
    dv = synthetic.synthetic_depth_values(1).to(DEV)
    gt, mask = _targets(gold)
    with golden_rot(model):
        st1 = fmt_train(model, leaves["stage1"])
        st2, st3 = pathway_train(model, st1, leaves["stage2"], leaves["stage3"])
        outputs = depth_stages_forward_train(model, {"stage1": st1, "stage2": st2, "stage3": st3}, proj, dv,
                                             (H, H * 5 // 4))
        terms = hip_loss.focal_loss_bld(outputs, gt, mask, torch.tensor([float(gold["f_interval"])]),
                                        dlossw=[1.0, 1.0, 1.0])
        terms[0].backward()
    torch.cuda.synchronize()
    _check_outputs(gold, "f", outputs, terms, exact["f"][2])
    got = {n: p.grad.detach().cpu().numpy() for n, p in model.named_parameters() if p.grad is not None}
    _judge(gold, exact["f"], "f", got)
    ref_fg = exact["f"][1]
    for k in STAGES:
        g = leaves[k].grad.detach().cpu().numpy()
        for v in range(N):
            e = _rel(g[v], ref_fg[f"{v}_{k}"])
            f32 = _rel(gold[f"f_featgrad_{v}_{k}"], ref_fg[f"{v}_{k}"])
            assert e <= max(1e-4, 3.0 * f32), (k, v, e, f32)
    _check_buffers(gold, "f", model)


@pytest.mark.parametrize("loss_impl", ["hip", "reference_torch_ops"])
def test_train_sample_unchanged_body_vs_reference(gold, exact, loss_impl):
    """finetune.py:144-168 on the drop-in model (FeatureNet + DCN backward included)."""
    from oracle import loss_ref
    from transmvsnet_amd import loss as hip_loss
    from transmvsnet_amd import synthetic
    from transmvsnet_amd.train import FlatAdam
    focal_loss_bld = hip_loss.focal_loss_bld if loss_impl == "hip" else loss_ref.focal_loss_bld
    model = _model()
    optimizer = FlatAdam([p for p in model.parameters()], lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4)
    imgs = synthetic.synthetic_images(N, H, H * 5 // 4, seed=0).to(DEV)
    proj = synthetic.synthetic_cameras(N, H, H * 5 // 4, seed=1)
    dv = synthetic.synthetic_depth_values(1).to(DEV)
    depth_gt_ms, mask_ms = _targets(gold)
    interval = torch.tensor([float(gold["i_interval"])], device=DEV)
    with golden_rot(model):
        # ---- the reference's train_sample body (finetune.py:145-168)
        model.train()
        optimizer.zero_grad()
        outputs = model(imgs, proj, dv)
        loss, depth_loss, epe, less1, less3 = focal_loss_bld(outputs, depth_gt_ms, mask_ms, interval,
                                                             dlossw=[1.0, 1.0, 1.0])
        loss.backward()
        grads = {n: p.grad.detach().cpu().numpy().copy() for n, p in model.named_parameters() if p.grad is not None}
        optimizer.step()
    torch.cuda.synchronize()
    _check_outputs(gold, "i", outputs, (loss, depth_loss, epe, less1, less3), exact["i"][2])
    _judge(gold, exact["i"], "i", grads)
    _check_buffers(gold, "i", model)
    # the step moved every parameter that has a gradient, and eval mode sees the new weights
    model.eval()
    with torch.no_grad():
        out = model(imgs, proj, dv)
    assert torch.isfinite(out["depth"]).all()


def test_flat_adam_accumulates_two_backwards_and_invalidates_inference_cache():
    """gradients accumulated over two backward passes before step() (no zero_grad between),
    step() twice, and an eval forward after the step sees the stepped weights (packed-weight caches
    keyed on parameter versions)."""
    from transmvsnet_amd import TransMVSNet, synthetic
    from transmvsnet_amd.train import FlatAdam
    torch.manual_seed(0)
    m = _model()
    params = [p for n, p in m.named_parameters() if n.startswith("cost_regularization.0.")]
    ref_params = [p.detach().clone().requires_grad_() for p in params]
    opt = FlatAdam(params, lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-4)
    ref_opt = torch.optim.Adam(ref_params, lr=1e-2, betas=(0.9, 0.999), weight_decay=1e-4)
    # no zero_grad anywhere: after the first step the .grad tensors are views into FlatAdam's flat
    # buffer, and the next "backwards" accumulate into them in place (two per step here)
    for step in range(3):
        for rep in range(2):
            g = [torch.randn_like(p) for p in params]
            for p, gg in zip(params, g):
                if p.grad is None:
                    p.grad = gg.clone()
                else:
                    p.grad.add_(gg)
            for p, gg in zip(ref_params, g):
                p.grad = gg.clone() if p.grad is None else p.grad + gg
        opt.step()
        ref_opt.step()
    opt.zero_grad()
    for p, r in zip(params, ref_params):
        assert float((p.detach() - r.detach()).abs().max()) < 1e-6
    # eval forward after the step == a model freshly loaded with the stepped weights
    sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
    fresh = TransMVSNet(ndepths=list(ND))
    fresh.load_state_dict(sd, strict=True)
    fresh = fresh.to(DEV).eval()
    m.eval()
    feats = synthetic.synthetic_features(N, H, H * 5 // 4, seed=2)
    proj = synthetic.synthetic_cameras(N, H, H * 5 // 4, seed=1)
    dv = synthetic.synthetic_depth_values(1).to(DEV)
    fd = [{k: v.to(DEV) for k, v in f.items()} for f in feats]
    with torch.no_grad():
        a = fresh.forward_features(fd, proj, dv, (H, H * 5 // 4))
        b = m.forward_features(fd, proj, dv, (H, H * 5 // 4))
        # a second step with no forward in between, then eval again: still the current weights
        for p in params:
            p.grad = torch.randn_like(p)
        opt.step()
        sd2 = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
        fresh.load_state_dict(sd2, strict=True)
        c = fresh.forward_features(fd, proj, dv, (H, H * 5 // 4))
        d = m.forward_features(fd, proj, dv, (H, H * 5 // 4))
    torch.cuda.synchronize()
    assert torch.equal(a["prob_volume"], b["prob_volume"])
    assert torch.equal(c["prob_volume"], d["prob_volume"])
    assert not torch.equal(a["prob_volume"], c["prob_volume"])


def test_train_sample_hip_graph_replay_equals_eager(gold):
    """The same train_sample body captured once as a HIP graph (train.TrainStepGraph, bench.py's
    training timing) and replayed: one eager step, an eval forward (builds the inference caches), two
    replays, an eval forward, and one more eager step leave the parameters, Adam moments and BatchNorm
    running statistics where four eager steps leave them (within 1e-5 of each quantity's max: the
    DCN's beyond-window corners use fp32 atomics, so not bitwise). Also: Adam's step number after
    the replays is 4 (the eager step after a capture uses the device counter), and the eval forward
    after the replays equals a fresh model's built from the same state_dict bit for bit (the replays
    invalidated the inference caches keyed on parameter versions)."""
    from transmvsnet_amd import loss as hip_loss
    from transmvsnet_amd import synthetic
    from transmvsnet_amd import train as tr
    imgs = synthetic.synthetic_images(N, H, H * 5 // 4, seed=0).to(DEV)
    proj = synthetic.synthetic_cameras(N, H, H * 5 // 4, seed=1)
    dv = synthetic.synthetic_depth_values(1).to(DEV)
    depth_gt_ms, mask_ms = _targets(gold)
    interval = torch.tensor([float(gold["i_interval"])])  # host (no device read inside the graph)
    runs = []
    for graphed in (False, True):
        model = _model()
        opt = tr.FlatAdam([p for p in model.parameters()], lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4)

        def body():
            model.train()
            opt.zero_grad()
            outputs = model(imgs, proj, dv)
            loss = hip_loss.focal_loss_bld(outputs, depth_gt_ms, mask_ms, interval, dlossw=[1.0, 1.0, 1.0])[0]
            loss.backward()
            opt.step()

        def eval_prob(m):
            m.eval()
            with torch.no_grad(), golden_rot(m):
                return m(imgs, proj, dv)["stage3"]["prob_volume"].clone()
        with golden_rot(model):
            body()
            eval_prob(model)  # the inference caches now hold step 1's weights
            torch.cuda.synchronize()
            if graphed:
                graph = tr.TrainStepGraph(body, model)  # captured, not run
                for _ in range(2):
                    graph.replay()
                torch.cuda.synchronize()
                graph.check_flags()
            else:
                for _ in range(2):
                    body()
            ev = eval_prob(model)
            fresh = _model()
            fresh.load_state_dict(model.state_dict())
            assert torch.equal(ev, eval_prob(fresh)), "eval forward used stale packed weights"
            body()  # an eager step after the replays: Adam step 4
        torch.cuda.synchronize()
        assert opt.step_count == 4, opt.step_count
        bufs = {n: b.detach().clone() for n, b in model.named_buffers() if "running" in n}
        runs.append((opt.flat.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), bufs))
    (fa, ma, va, ba), (fb, mb, vb, bb) = runs
    for a, b, tag in ((fa, fb, "params"), (ma, mb, "exp_avg"), (va, vb, "exp_avg_sq")):
        err = float((a - b).abs().max() / a.abs().max())
        assert err < 1e-5, (tag, err)
    for n in ba:
        err = float((ba[n] - bb[n]).abs().max() / max(float(ba[n].abs().max()), 1e-30))
        assert err < 1e-5, (n, err)
