"""transmvsnet_amd.bn_running: the batched running-statistics update equals nn.BatchNorm's sequential
per-call updates (a module called once per view, G calls, momentum 0.1) within fp32 re-association."""
import torch

from transmvsnet_amd.bn_running import update_running_stats


def test_closed_form_equals_sequential_calls():
    torch.manual_seed(0)
    for g, c in ((1, 8), (3, 16), (5, 32)):
        seq = torch.nn.BatchNorm2d(c, momentum=0.1)
        fast = torch.nn.BatchNorm2d(c, momentum=0.1)
        rm0, rv0 = torch.randn(c), torch.rand(c) + 0.5
        for bn in (seq, fast):
            bn.running_mean.copy_(rm0)
            bn.running_var.copy_(rv0)
        xs = [torch.randn(1, c, 7, 9) * (v + 1) + v for v in range(g)]
        seq.train()
        for x in xs:  # the reference: one call per view
            seq(x)
        means = torch.stack([x.mean((0, 2, 3)) for x in xs])
        vars_ = torch.stack([x.var((0, 2, 3), unbiased=False) for x in xs])
        update_running_stats([(fast, means, vars_, 63)], 0.1)
        assert torch.allclose(fast.running_mean, seq.running_mean, rtol=1e-6, atol=1e-6)
        assert torch.allclose(fast.running_var, seq.running_var, rtol=1e-6, atol=1e-6)
        assert int(fast.num_batches_tracked) == int(seq.num_batches_tracked) == g
