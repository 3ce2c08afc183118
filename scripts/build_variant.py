"""Build an experimental copy of the library with extra compile flags (A/B kernel experiments).

    python scripts/build_variant.py NAME -DFLAG=1 ...   ->  variants/NAME/libtransmvs_hip.so

Load it with TMVS_LIB_PATH=variants/NAME/libtransmvs_hip.so (transmvsnet_amd/_lib.py).
"""
import concurrent.futures as cf
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from transmvsnet_amd import build as B  # noqa: E402

name, extra = sys.argv[1], sys.argv[2:]
out = os.path.join(B.ROOT, "variants", name)
os.makedirs(out, exist_ok=True)


def comp(src):
    o = os.path.join(out, src.replace(".hip", ".o"))
    r = subprocess.run([B.HIPCC, *B.CFLAGS, *extra, "-c", os.path.join(B.CSRC, src), "-o", o], capture_output=True,
                       text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    return o


with cf.ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(comp, B.SOURCES))
lib = os.path.join(out, "libtransmvs_hip.so")
subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-fno-gpu-rdc", "-o", lib, *objs], check=True)
print(lib)
