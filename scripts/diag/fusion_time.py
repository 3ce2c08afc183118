"""Depth-map fusion at DTU test size: V views of 864x1152 (synthetic plane scene, tests/_fusion_scene.py),
tmvs_fusibile per reference camera (HIP events), the whole fusion.fuse (kernel + compaction), and
the CPU oracle on one reference camera for scale. Usage: fusion_time.py [V]"""
import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
from tests._fusion_scene import make_scene
from oracle import fusion_ref
from transmvsnet_amd import _lib, fusion, ops
V = int(sys.argv[1]) if len(sys.argv) > 1 else 49
H, W = 864, 1152
t0 = time.time()
rgbd, packs, dicts, _ = make_scene(v=V, h=H, w=W, seed=1)
print(f"scene {V}x{H}x{W} built in {time.time() - t0:.1f} s", flush=True)
rg = torch.from_numpy(rgbd).cuda()
cams = torch.from_numpy(packs).cuda()
lib = _lib.load()
coord = torch.zeros(H, W, 4, device="cuda")
tex = torch.zeros(H, W, 4, device="cuda")
ts = []
for rep in range(3):
    for ref in range(V):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.check(lib.tmvs_fusibile(rg.data_ptr(), cams.data_ptr(), V, H, W, ref, 3, 0.25, coord.data_ptr(),
                                     tex.data_ptr(), ops._stream()), "tmvs_fusibile")
        e1.record()
        torch.cuda.synchronize()
        if rep > 0:
            ts.append(e0.elapsed_time(e1))
k_ms = float(np.mean(ts))
t0 = time.perf_counter()
xs, tt = fusion.fuse(rg, packs)
torch.cuda.synchronize()
fuse_ms = (time.perf_counter() - t0) * 1e3
t0 = time.perf_counter()
wr, cx, ct = fusion_ref.fusibile_ref(rgbd, dicts, 0)
cpu_s = time.perf_counter() - t0
# bytes actually touched per launch: the reference view's row + 4 texels x 16 B per sampled view
print(f"tmvs_fusibile: {k_ms * 1e3:.1f} us per reference camera ({H}x{W}, {V} views); fuse() all {V} cameras "
      f"incl. compaction {fuse_ms:.1f} ms, {len(xs)} points; CPU oracle (numpy, float64) one camera "
      f"{cpu_s:.2f} s -> {cpu_s * 1e3 / k_ms:.0f}x")
