"""Build the HIP extension in-tree: transmvsnet_amd/libtransmvs_hip.so (gfx950 only).

    python -m transmvsnet_amd.build [--force]

One hipcc invocation per translation unit (parallel), then one link. No torch headers:
the library is a plain C-ABI (include/transmvs.h) loaded through ctypes.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "libtransmvs_hip.so")
ARCH = os.environ.get("TMVS_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["host.hip", "glue.hip", "warp_corr.hip", "costreg.hip", "fmt.hip", "pathway.hip", "pipeline.hip", "featurenet.hip",
           "conv2d.hip", "fusion.hip", "loss.hip", "costreg_train.hip", "pw_train.hip", "pathway_train.hip",
           "fmt_train.hip", "optim.hip", "featurenet_train.hip"]
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fno-gpu-rdc",
          "-Wall", "-Wno-unused-function", "-I", os.path.join(ROOT, "include")]


def _newer(src_paths, dst):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(p) > t for p in src_paths)


def _compile(src, force):
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, src.replace(".hip", ".o"))
    deps = [s, os.path.join(ROOT, "include", "transmvs.h")] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")]
    if not force and not _newer(deps, o):
        return o, None
    cmd = [HIPCC, *CFLAGS, "-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return o, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return o, None


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        results = list(ex.map(lambda s: _compile(s, force), SOURCES))
    errors = [e for _, e in results if e]
    if errors:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errors))
    objs = [o for o, _ in results]
    if force or _newer(objs, LIB):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fno-gpu-rdc", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
