"""Capture the bench's C5 training step (full | features) as a HIP graph and print the full traceback
of the first operation that is not capturable (diagnostic, GPU box)."""
import os
import sys
import traceback

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch

import bench

kind = sys.argv[1]
dev = torch.device("cuda", 0)
full_step, features_step, _ = bench.train_steps(dev)
fn = full_step if kind == "full" else features_step
side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    fn()
torch.cuda.current_stream(dev).wait_stream(side)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g):
        fn()
    print(kind, "captured", flush=True)
except Exception:
    traceback.print_exc()
