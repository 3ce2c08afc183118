"""Multi-process pieces of the GPU path that need no multi-GPU box (needs an MI355X; -m gpu).

* FlatAdam's DDP step (finetune.py:358-362 wraps the model in DDP; its gradient sync is
  FlatAdam.allreduce = one all-reduce of the flat gradient buffer, then the HIP Adam step): two
  ranks on gloo (all-reduce of device tensors), both on cuda:0, different gradients per rank. Every
  rank must end with the rank-mean gradient and bitwise identical parameters and moments, equal
  to one process stepping with that mean gradient.
* The view-sharded forward (models/TransMVSNet.py:74-93 split over ranks, one all-reduce per
  stage) captured as one HIP graph: on a one-rank RCCL group with the collective forced
  (ViewShard.always_reduce), replay == eager bit for bit, and both equal the unsharded forward
  within the partial-sum tolerance.
Ranks run as spawned processes (a fresh interpreter each; the test process's own GPU state is not
forked), rendezvous over a file store.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
SHAPES = [(8, 1, 3, 3, 3), (16,), (64, 32)]


def _store():
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="tmvs_gpu_dist_"), "store")


def _grads(rank):
    g = torch.Generator().manual_seed(300 + rank)
    return [torch.randn(s, generator=g) * 0.1 for s in SHAPES]


def _init_params():
    g = torch.Generator().manual_seed(299)
    return [torch.randn(s, generator=g) for s in SHAPES]


def _adam_worker(rank, world, store, q):
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=store, rank=rank, world_size=world)
    try:
        from transmvsnet_amd.train import FlatAdam
        ps = [torch.nn.Parameter(t.cuda()) for t in _init_params()]
        opt = FlatAdam(ps, lr=1e-3, weight_decay=1e-4)
        for _ in range(2):
            opt.zero_grad()
            for p, gr in zip(ps, _grads(rank)):
                p.grad = gr.cuda()
            opt.allreduce()
            opt.step()
        torch.cuda.synchronize()
        q.put((rank, opt.grad_flat.cpu().numpy().copy(), opt.flat.cpu().numpy().copy(),
               opt.exp_avg.cpu().numpy().copy(), opt.exp_avg_sq.cpu().numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_flat_adam_allreduce_step_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = _store()
    procs = [ctx.Process(target=_adam_worker, args=(r, world, store, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, *arrs = q.get(timeout=240)
        res[r] = arrs
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # one process stepping with the rank-mean gradient (sum of the two, then / 2: the same roundings)
    from transmvsnet_amd.train import FlatAdam
    ps = [torch.nn.Parameter(t.cuda()) for t in _init_params()]
    opt = FlatAdam(ps, lr=1e-3, weight_decay=1e-4)
    mean = [(a + b) / 2 for a, b in zip(_grads(0), _grads(1))]
    for _ in range(2):
        opt.zero_grad()
        for p, gr in zip(ps, mean):
            p.grad = gr.cuda()
        opt.step()
    torch.cuda.synchronize()
    expect = [opt.grad_flat.cpu().numpy(), opt.flat.cpu().numpy(), opt.exp_avg.cpu().numpy(),
              opt.exp_avg_sq.cpu().numpy()]
    for r in range(world):
        for i, tag in enumerate(("grad", "params", "exp_avg", "exp_avg_sq")):
            np.testing.assert_array_equal(res[r][i], res[0][i], err_msg=f"rank {r} {tag} differs from rank 0")
            np.testing.assert_array_equal(res[r][i], expect[i], err_msg=f"rank {r} {tag} vs one process with the mean")


def _views_graph_worker(store, q):
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=store, rank=0, world_size=1, device_id=dev)
    try:
        from transmvsnet_amd import TransMVSNet, synthetic
        from transmvsnet_amd.distributed import ViewShard
        H, W, N = 256, 320, 4
        model = TransMVSNet().eval()
        model.load_state_dict(synthetic.synthetic_state_dict(synthetic.state_dict_shapes(model), seed=0, sharpen=100.0))
        model = model.to(dev)
        feats = {k: v.to(dev) for k, v in synthetic.stacked_features(N, H, W, seed=2).items()}
        proj = synthetic.synthetic_cameras(N, H, W, seed=1)
        dv = synthetic.synthetic_depth_values(1).to(dev)
        shard = ViewShard(0, 1, N - 1, always_reduce=True)
        with torch.no_grad():
            full = model.forward_features(feats, proj, dv, (H, W))
            eager = model.forward_features(feats, proj, dv, (H, W), view_shard=shard)
            torch.cuda.synchronize()
            eager = {s: {k: eager[s][k].clone() for k in ("depth", "prob_volume")} for s in ("stage1", "stage2", "stage3")}
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                g_out = model.forward_features(feats, proj, dv, (H, W), view_shard=shard)
            for _ in range(2):
                graph.replay()
            torch.cuda.synchronize()
        res = {"n_allreduce": len(shard.comm_bytes)}
        for s in ("stage1", "stage2", "stage3"):
            res[s] = {
                "replay_equal": bool(torch.equal(g_out[s]["prob_volume"], eager[s]["prob_volume"])
                                     and torch.equal(g_out[s]["depth"], eager[s]["depth"])),
                "prob_vs_unsharded": float((eager[s]["prob_volume"] - full[s]["prob_volume"]).abs().max()),
                "depth_mean_vs_unsharded": float((eager[s]["depth"] - full[s]["depth"]).abs().mean()),
            }
        q.put(res)
    finally:
        dist.destroy_process_group()


def test_view_sharded_forward_graph_capture_equals_eager_rccl():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_views_graph_worker, args=(_store(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    print(res)
    assert res["n_allreduce"] == 3  # one collective per stage (captured in the graph)
    for s in ("stage1", "stage2", "stage3"):
        assert res[s]["replay_equal"], (s, res)
        # the partial + finalize path re-associates the view sum (tests/test_distributed.py's bar)
        assert res[s]["prob_vs_unsharded"] < 2e-4 and res[s]["depth_mean_vs_unsharded"] <= 1e-4, (s, res)
