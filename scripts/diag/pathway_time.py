"""The FMT pathway launches alone (no concurrent stage-1 kernels), DTU full size, HIP-event medians.

    python scripts/diag/pathway_time.py [REPS]          (TMVS_LIB_PATH selects a library variant)
Prints the stage-2 (32 -> 16, `tmvs_fmt_pathway` cc=32) and stage-3 (16 -> 8) per-launch medians.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from transmvsnet_amd import TransMVSNet, ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = TransMVSNet().eval()
prep = m._prepared(dev)
nv, h, w = 5, 216, 288
st1 = torch.randn(nv, h, w, 32, device=dev)
s2 = torch.randn(nv, 16, 2 * h, 2 * w, device=dev)
s3 = torch.randn(nv, 8, 4 * h, 4 * w, device=dev)


def med(fn):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


out2 = ops.fmt_pathway(st1, s2, prep["red1"], prep["sm1"])
t2 = med(lambda: ops.fmt_pathway(st1, s2, prep["red1"], prep["sm1"]))
t3 = med(lambda: ops.fmt_pathway(out2, s3, prep["red2"], prep["sm2"]))
print(f"pathway {os.environ.get('TMVS_LIB_PATH', 'default')}: stage 2 {t2:.1f} us, stage 3 {t3:.1f} us, "
      f"stage-2 checksum {float(out2.double().sum()):.9e}")
