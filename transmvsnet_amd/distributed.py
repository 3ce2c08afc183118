"""View-sharded cost volume across ranks (one process per GPU, RCCL over xGMI).

The only cross-view reduction of the hot path is DepthNet's view aggregation
(models/TransMVSNet.py:72-93):

    sim = (1e-5 + sum_v w_v) ^-1 * sum_v w_v * sim_v

Each rank owns a contiguous slice of the source views. It runs FMT/pathway for the reference
view plus its own source views only (a source view's FMT depends on the reference view and
itself, models/FMT.py:160-176), builds the PARTIAL cost volume of its views
(tmvs_warp_corr with TMVS_WARP_PARTIAL: sum w*sim and sum w, written into one packed buffer),
and one all-reduce of that buffer per stage gives every rank the full aggregate, finished by
tmvs_aggregate_finalize. CostRegNet / softmax then run replicated (identical inputs, identical
outputs on every rank). Stage-1 view weights stay rank-local: later stages only read the
weights of the rank's own views.

Summation order differs from the reference's sequential loop (per-rank partial sums, then the
ring sum), so results match the single-GPU path within fp32 rounding, not bit-for-bit; the
test tolerance is in tests/test_distributed.py.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch
import torch.distributed as dist


def partition_views(n_src: int, world: int, rank: int) -> List[int]:
    """Contiguous, balanced split of source views 0..n_src-1; ranks beyond n_src own none."""
    base, extra = divmod(n_src, world)
    start = rank * base + min(rank, extra)
    count = base + (1 if rank < extra else 0)
    return list(range(start, start + count))


def view_groups(world: int, n_src: int) -> tuple:
    """Replica x view-shard layout of `world` ranks for n_src source views: the view-shard group size g
    is the largest divisor of world that is <= n_src (more ranks than source views would leave some
    idle), so world = replicas x g; group r holds ranks r*g .. r*g + g - 1 and computes its own depth
    maps. -> (g, replicas)."""
    g = max(d for d in range(1, min(world, n_src) + 1) if world % d == 0)
    return g, world // g


def make_view_shard(rank: int, world: int, n_src: int, **kw) -> "ViewShard":
    """This rank's ViewShard in the replica x view-shard layout (view_groups). Every rank creates every
    group (torch.distributed.new_group is collective), in the same order."""
    g, replicas = view_groups(world, n_src)
    group = None
    if replicas > 1:
        groups = [dist.new_group(list(range(r * g, (r + 1) * g))) for r in range(replicas)]
        group = groups[rank // g]
    shard = ViewShard(rank % g, g, n_src, group=group, **kw)
    shard.replica = rank // g
    shard.replicas = replicas
    return shard


class ViewShard:
    """Source-view sharding for TransMVSNet.forward_features(view_shard=...).

    partial_fn(fs, rows, hyp, stage, view_w, pw, sim_out, wsum_out) -> new stage-1 view
    weights (or None) and finalize_fn(sim_sum, w_sum) default to the HIP ops; tests inject
    CPU restatements to check the sharding/reduction protocol on the gloo backend.
    """

    def __init__(self, rank: int, world: int, n_src: int, group=None,
                 partial_fn: Optional[Callable] = None, finalize_fn: Optional[Callable] = None,
                 always_reduce: bool = False):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.rank, self.world, self.n_src, self.group = rank, world, n_src, group
        self.src_views = partition_views(n_src, world, rank)
        self._partial = partial_fn or _hip_partial
        self._finalize = finalize_fn or _hip_finalize
        self.replica, self.replicas = 0, 1  # make_view_shard: this rank's replica group, and their count
        self.timer = None       # optional begin(name)/end(token) around each collective (bench.py)
        # issue the all-reduce even at world 1 (a one-rank group: the collective is a copy) -- tests use
        # it to capture the collective in a HIP graph on a single GPU
        self.always_reduce = always_reduce
        self.comm_bytes = []    # bytes of each all-reduce issued, in order (3 per forward)

    @property
    def local_views(self) -> List[int]:
        """Indices into the full view list (0 = reference) this rank processes."""
        return [0] + [1 + v for v in self.src_views]

    def select_features(self, feats: dict) -> dict:
        """{stage: [B,N,C,h,w]} -> the reference + own source views."""
        idx = self.local_views
        if len(idx) == feats["stage1"].shape[1]:
            return feats
        return {k: v[:, idx].contiguous() for k, v in feats.items()}

    def select_rows(self, rows):
        """proj rows [B,V,12] (source views) -> own source views."""
        return rows[:, self.src_views]

    def cost_volume(self, fs, rows, hyp, stage, view_w, pw, rot_order="auto"):
        """Full aggregated similarity [1,D,h,w] on every rank + this rank's stage-1 view weights.

        fs: [1+n_local, h, w, C] NHWC (reference first); rows: [1, n_local, 12] host array.
        """
        d, h, w = hyp.shape[1], hyp.shape[2], hyp.shape[3]
        # the partial kernels overwrite sim_sum / w_sum; only a rank without source views contributes zeros
        buf = torch.empty(1, d + 1, h, w, device=hyp.device, dtype=torch.float32)
        sim_sum, w_sum = buf[:, :d], buf[:, d]
        new_vw = view_w
        if self.src_views:
            new_vw = self._partial(fs, rows, hyp, stage, view_w, pw, sim_sum, w_sum, rot_order=rot_order)
        else:
            buf.zero_()
        self.allreduce(buf)
        sim = buf[:, :d]
        self._finalize(sim, buf[:, d])
        return sim, (new_vw if stage == 0 else view_w)

    def allreduce(self, buf: torch.Tensor) -> None:
        """The stage's one collective. Graph-capturable on RCCL: `bench.py --mode views` captures the
        whole view-sharded step (FMT, pathway, partial volumes, these all-reduces, finalize,
        CostRegNet) as one HIP graph and replays it per step, like replica mode."""
        if self.world > 1 or self.always_reduce:
            tok = self.timer.begin("rccl_all_reduce") if self.timer is not None else None
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
            if tok is not None:
                self.timer.end(tok)
            if len(self.comm_bytes) < 3:
                self.comm_bytes.append(buf.numel() * buf.element_size())


def _hip_partial(fs, rows, hyp, stage, view_w, pw, sim_out, wsum_out, rot_order="auto"):
    from . import ops
    ref = fs[0:1]
    src = fs[1:].unsqueeze(0)
    if stage == 0:
        _, _, vw = ops.warp_corr(ref, src, rows, hyp, pw_params=pw, partial=True, sim_out=sim_out, wsum_out=wsum_out,
                                 rot_order=rot_order)
        return vw
    ops.warp_corr(ref, src, rows, hyp, view_w_in=view_w, vw_shift=stage, partial=True, sim_out=sim_out,
                  wsum_out=wsum_out, rot_order=rot_order)
    return None


def _hip_finalize(sim_sum, w_sum):
    from . import ops
    ops.aggregate_finalize(sim_sum, w_sum)
