"""Run ONE kind of the bench's C5 training step alone (for rocprofv3 --kernel-trace --stats):
    python scripts/diag/train_prof.py full|features STEPS [graph]
(1 warm-up step first; with `graph` the step is captured once and replayed STEPS times; diagnostic,
GPU box)"""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch

import bench

kind, steps = sys.argv[1], int(sys.argv[2])
dev = torch.device("cuda", 0)
full_step, features_step, _ = bench.train_steps(dev)
fn = full_step if kind == "full" else features_step
fn()
torch.cuda.synchronize()
if len(sys.argv) > 3 and sys.argv[3] == "graph":
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    fn = g.replay
for i in range(steps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{kind} step {i}: {e0.elapsed_time(e1):.3f} ms", flush=True)
