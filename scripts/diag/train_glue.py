"""Which Python call sites launch torch's own kernels (copies, fills, index, elementwise) inside the C5
training step: one eager full_step (bench._train_setup) under torch.profiler, aten ops that launch device
work grouped by op and the innermost transmvsnet_amd / bench frame of their Python stack.

    python scripts/diag/train_glue.py [top]
"""
import collections
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch  # noqa: E402

import bench  # noqa: E402

OPS = ("aten::copy_", "aten::zero_", "aten::fill_", "aten::index", "aten::index_put_", "aten::cat", "aten::add_",
       "aten::mul", "aten::add", "aten::sub", "aten::div", "aten::clone", "aten::contiguous", "aten::zeros",
       "aten::ones", "aten::sum", "aten::max", "aten::stack", "aten::to", "aten::_to_copy", "aten::empty_like",
       "aten::where", "aten::lerp_", "aten::addcmul_", "aten::sqrt", "aten::mul_", "aten::div_", "aten::_foreach_copy_",
       "aten::_foreach_zero_", "aten::_foreach_add_", "aten::copy")


def main():
    top = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    torch.cuda.set_device(0)
    full_step, _, _ = bench._train_setup(torch.device("cuda", 0))
    full_step()
    full_step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=False) as prof:
        full_step()
        torch.cuda.synchronize()
    counts = collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        site = "?"
        for fr in (ev.stack or []):
            if "transmvsnet_amd" in fr or "bench.py" in fr:
                site = fr.split("repo/")[-1]
                break
        counts[(ev.name, site)] += 1
    print(f"{sum(counts.values())} aten calls of the listed kinds in one step; top call sites:")
    for (name, site), n in counts.most_common(top):
        print(f"{n:6d}  {name:24s} {site}")


if __name__ == "__main__":
    main()
