"""Which Python call sites issue torch's own device ops (copies, fills, index, elementwise) in one eager C5
training step (bench._train_setup's full_step): a TorchDispatchMode records every aten op with the innermost
transmvsnet_amd / bench frame of the Python stack (forward, loss and the custom Functions' backward).
Ops on host tensors and ops that launch no device work (views, metadata) are skipped.

    python scripts/diag/train_glue2.py [top]
"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch  # noqa: E402
import torch.utils._pytree  # noqa: E402,F401
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402

SKIP = ("view", "reshape", "expand", "permute", "transpose", "unsqueeze", "squeeze", "select", "slice", "detach",
        "alias", "as_strided", "t.default", "_unsafe_view", "empty", "set_", "is_", "size", "stride", "numel", "dim",
        "split", "unbind", "chunk", "lift_fresh", "_to_copy.default_host", "item", "_local_scalar_dense", "resize_")


class Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.counts = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        on_gpu = any(isinstance(a, torch.Tensor) and a.is_cuda
                     for a in torch.utils._pytree.tree_flatten((args, kwargs or {}))[0])
        if on_gpu and not any(s in name for s in SKIP):
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                f = fr.filename
                if ("transmvsnet_amd" in f or "bench.py" in f) and "_python_dispatch" not in f:
                    site = f"{f.split('repo/')[-1]}:{fr.lineno} ({fr.name})"
                    break
            self.counts[(name, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    top = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    torch.cuda.set_device(0)
    full_step, _, _ = bench._train_setup(torch.device("cuda", 0))
    full_step()
    full_step()
    torch.cuda.synchronize()
    rec = Rec()
    with rec:
        full_step()
    torch.cuda.synchronize()
    print(f"{sum(rec.counts.values())} aten ops with device work in one step; top call sites:")
    for (name, site), n in rec.counts.most_common(top):
        print(f"{n:6d}  {name:40s} {site}")


if __name__ == "__main__":
    main()
