"""C5 full training step (bench._train_setup) captured as one HIP graph and replayed REPS times with a 50-ms
host gap between replays, for rocprofv3 --kernel-trace; scripts/diag/train_graph_table.py then splits the
trace at the gaps and tables the last replay's kernels.

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 scripts/diag/train_graph_prof.py [REPS]
"""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import torch  # noqa: E402

import bench  # noqa: E402
from transmvsnet_amd import train as _train  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
full_step, _, m = bench._train_setup(dev)
side = torch.cuda.Stream(dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    full_step()
torch.cuda.current_stream(dev).wait_stream(side)
torch.cuda.synchronize()
g = _train.TrainStepGraph(full_step, m)
torch.cuda.synchronize()
ts = []
for _ in range(reps):
    time.sleep(0.05)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
print("replay ms:", " ".join(f"{t:.2f}" for t in ts), flush=True)
