"""CPU dry run of a GPU diag script's Python side (argument shapes, wrapper checks, control flow) before
spending a GPU call on it: patches transmvsnet_amd.ops so wrappers validate their arguments as on the GPU
but launch nothing (every tmvs_* entry returns OK, workspaces are small), and HIP events / synchronize
into no-ops. Outputs are uninitialised.  Usage: TMVS_DRYRUN=1 python scripts/diag/dryrun.py SCRIPT [args]
(the scripts pick the CPU device when TMVS_DRYRUN is set)."""
import os
import runpy
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["TMVS_DRYRUN"] = "1"
from transmvsnet_amd import _lib, ops  # noqa: E402


class _FakeLib:
    def __getattr__(self, name):
        return (lambda *a: 4096) if name.endswith("_workspace") else (lambda *a: 0)


def _dev(t, name):
    if t is None:
        return
    if t.dtype != torch.float32 or not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous float32")


class _Event:
    def __init__(self, *a, **k):
        pass

    def record(self, *a):
        pass

    def elapsed_time(self, other):
        return 0.0


ops._dev = _dev
ops._lib_h = lambda: _FakeLib()
ops._stream = lambda: None
_lib.check = lambda rc, name: None
torch.cuda.Event = _Event
torch.cuda.synchronize = lambda *a: None
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
