"""Run bench.train_timing (C5 DepthNet-stage training step) alone, for rocprofv3 --stats."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch

import bench

torch.cuda.set_device(0)
print(bench.train_timing(int(os.environ.get("STEPS", "3")), torch.device("cuda", 0), 1))
