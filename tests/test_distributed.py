"""View sharding (transmvsnet_amd.distributed) on the gloo backend, world_size 2 and 3, CPU.

The HIP partial cost volume is replaced by a restatement of the reference's per-view loop
(models/TransMVSNet.py:58-93) restricted to the rank's views, so this checks the sharding and
reduction protocol: every rank must end with the full-view aggregate of oracle.build_cost_volume.
Tolerance: 1e-6 abs on O(1e-1) similarities (partial sums re-associate the view sum).
"""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import transmvs_ref as oracle
from transmvsnet_amd import synthetic
from transmvsnet_amd.distributed import ViewShard, partition_views
from tests._util import golden_state_dict

N_VIEWS, C, D, H, W = 5, 8, 8, 12, 16


def test_partition_views_covers_once():
    for n_src in (1, 2, 3, 4, 7):
        for world in (1, 2, 3, 4, 8):
            parts = [partition_views(n_src, world, r) for r in range(world)]
            flat = [v for p in parts for v in p]
            assert flat == list(range(n_src))
            sizes = [len(p) for p in parts]
            assert max(sizes) - min(sizes) <= 1


def test_select_features_and_rows():
    s = ViewShard(1, 2, 4)
    assert s.src_views == [2, 3] and s.local_views == [0, 3, 4]
    feats = {"stage1": torch.arange(5.).view(1, 5, 1, 1, 1).expand(1, 5, 2, 2, 2).contiguous()}
    out = s.select_features(feats)
    assert out["stage1"][0, :, 0, 0, 0].tolist() == [0., 3., 4.]
    import numpy as np
    rows = np.arange(4 * 12, dtype=np.float32).reshape(1, 4, 12)
    assert (s.select_rows(rows) == rows[:, 2:]).all()


def _inputs():
    g = torch.Generator().manual_seed(7)
    feats = [torch.randn(1, C, H, W, generator=g) for _ in range(N_VIEWS)]
    proj = synthetic.synthetic_cameras(N_VIEWS, H * 4, W * 4, seed=1)["stage1"]
    dv = torch.linspace(450.0, 900.0, D).view(1, D, 1, 1).expand(1, D, H, W).contiguous()
    return feats, proj, dv


def _oracle_partial(sd, feats, proj):
    """Factory: partial (sum w*sim, sum w) over a rank's source views, reference op order."""
    projs = torch.unbind(proj, 1)

    def partial(fs, rows, hyp, stage, view_w, pw, sim_out, wsum_out, views=None):
        ref = feats[0]
        vws = []
        sim_out.zero_()   # the HIP partial overwrites its outputs (ViewShard hands it uninitialised memory)
        wsum_out.zero_()
        for v in views:
            warped = oracle.homo_warping(feats[1 + v], oracle.compose_proj(projs[1 + v]),
                                         oracle.compose_proj(projs[0]), hyp)
            sim = (warped * ref.unsqueeze(2)).mean(1, keepdim=True)
            vw = oracle.pixelwise_net(sd, sim)
            sim_out += (sim * vw.unsqueeze(1))[:, 0]
            wsum_out += vw[:, 0]
            vws.append(vw)
        return torch.cat(vws, 1)
    return partial


def _finalize(sim_sum, w_sum):
    sim_sum.div_(1e-5 + w_sum.unsqueeze(1))


def _worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        sd = golden_state_dict()
        feats, proj, dv = _inputs()
        part = _oracle_partial(sd, feats, proj)
        shard = ViewShard(rank, world, N_VIEWS - 1, finalize_fn=_finalize)
        shard._partial = lambda *a, **k: part(*a, views=shard.src_views)
        sim, vw = shard.cost_volume(None, None, dv, 0, None, None)
        ref_sim, ref_vw = oracle.build_cost_volume(sd, feats, proj, dv)
        err = float((sim - ref_sim[:, 0]).abs().max())
        vw_err = 0.0
        if shard.src_views:
            vw_err = float((vw - ref_vw[:, shard.src_views]).abs().max())
        q.put((rank, err, vw_err, float(ref_sim.abs().max())))
    finally:
        dist.destroy_process_group()


def _free_port():
    """A file:// rendezvous in a fresh directory (no TCP port to race for when test files run in parallel)."""
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="tmvs_gloo_"), "store")


@pytest.mark.parametrize("world", [2, 3])
def test_view_sharded_cost_volume_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err, vw_err, scale in res:
        assert scale > 1e-3
        assert err <= 1e-6, (rank, err)
        assert vw_err == 0.0, (rank, vw_err)


def _grad_worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        from transmvsnet_amd.train import allreduce_gradients
        g = torch.Generator().manual_seed(100 + rank)
        params = [torch.nn.Parameter(torch.zeros(n)) for n in (5, 300, 7)]
        for p in params:
            p.grad = torch.randn(p.shape, generator=g)
        allreduce_gradients(params, bucket_bytes=1024)  # forces several buckets
        got = [p.grad.numpy().copy() for p in params]  # plain arrays: a queued tensor is shared by fd and dies with this process
        # the same sync on FlatAdam's single flat gradient buffer (its parameters are views of one buffer)
        from transmvsnet_amd.train import FlatAdam
        g = torch.Generator().manual_seed(100 + rank)
        params2 = [torch.nn.Parameter(torch.zeros(n)) for n in (5, 300, 7)]
        opt = FlatAdam(params2)
        for p in params2:
            p.grad = torch.randn(p.shape, generator=g)
        opt.allreduce()
        q.put((rank, got, [p.grad.numpy().copy() for p in params2]))
    finally:
        dist.destroy_process_group()


def test_allreduce_gradients_is_the_rank_mean():
    """train.allreduce_gradients (DDP's gradient sync) over gloo, world 2, multiple buckets; and
    FlatAdam.allreduce (one all-reduce of the flat gradient buffer)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    res = {r: g for r, g, _ in out}
    res_flat = {r: g for r, _, g in out}
    for p in procs:
        p.join(timeout=60)
    expect = []
    for n_i, n in enumerate((5, 300, 7)):
        acc = 0
        for r in range(world):
            gg = torch.Generator().manual_seed(100 + r)
            grads = [torch.randn(m, generator=gg) for m in (5, 300, 7)]
            acc = acc + grads[n_i]
        expect.append(acc / world)
    for r in range(world):
        for got, exp in zip(res[r], expect):
            torch.testing.assert_close(torch.from_numpy(got), exp, rtol=1e-6, atol=1e-6)
        for got, exp in zip(res_flat[r], expect):
            torch.testing.assert_close(torch.from_numpy(got), exp, rtol=1e-6, atol=1e-6)


def test_flat_adam_views():
    """FlatAdam (host side, no GPU): parameters keep their values and become views of one flat
    buffer; the gradients autograd leaves are gathered into the flat gradient (a missing one as
    zeros) and each .grad re-pointed at its slice; zero_grad drops them."""
    from transmvsnet_amd.train import FlatAdam
    ps = [torch.nn.Parameter(torch.randn(3, 4)), torch.nn.Parameter(torch.randn(7)), torch.nn.Parameter(torch.randn(2))]
    vals = [p.detach().clone() for p in ps]
    opt = FlatAdam(ps)
    assert opt.flat.numel() == 21
    for p, v in zip(ps, vals):
        assert torch.equal(p.detach(), v)
    assert ps[1].data_ptr() == opt.flat[12:].data_ptr()
    (ps[0].sum() * 2 + ps[1].sum()).backward()
    opt.allreduce()  # world 1: gathers only
    assert torch.equal(opt.grad_flat, torch.cat([torch.full((12,), 2.0), torch.ones(7), torch.zeros(2)]))
    assert ps[1].grad.data_ptr() == opt.grad_flat[12:].data_ptr()
    opt.zero_grad()
    assert all(p.grad is None for p in ps)


def test_view_groups_layout():
    from transmvsnet_amd.distributed import view_groups
    assert view_groups(8, 4) == (4, 2)
    assert view_groups(4, 4) == (4, 1)
    assert view_groups(2, 4) == (2, 1)
    assert view_groups(6, 4) == (3, 2)
    assert view_groups(5, 4) == (1, 5)
    assert view_groups(16, 10) == (8, 2)


def _hybrid_worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        from transmvsnet_amd.distributed import make_view_shard
        torch.set_num_threads(1)
        sd = golden_state_dict()
        feats, proj, dv = _inputs()
        feats, proj = feats[:3], proj[:, :3]  # 2 source views
        part = _oracle_partial(sd, feats, proj)
        shard = make_view_shard(rank, world, 2, finalize_fn=_finalize)
        shard._partial = lambda *a, **k: part(*a, views=shard.src_views)
        sim, _ = shard.cost_volume(None, None, dv, 0, None, None)
        ref_sim, _ = oracle.build_cost_volume(sd, feats, proj, dv)
        q.put((rank, shard.replica, shard.replicas, shard.src_views, float((sim - ref_sim[:, 0]).abs().max())))
    finally:
        dist.destroy_process_group()


def test_replica_by_view_shard_groups_gloo():
    """World 4 over 2 source views: 2 replica groups x 2 view shards (the layout bench.py
    --mode views uses when ranks outnumber source views); each group's all-reduce stays inside it and
    every rank gets the full aggregate."""
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hybrid_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = 2
    for rank, replica, replicas, views, err in res:
        assert replicas == world // g and replica == rank // g
        assert views == [rank % g], (rank, views)
        assert err <= 1e-6, (rank, err)
