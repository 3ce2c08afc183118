"""A/B variant of the library: recompile ONE translation unit with extra -D flags, link it with the
product objects into variants/NAME/libtransmvs_hip.so (load with TMVS_LIB_PATH=...).

    python scripts/build_variant.py NAME SOURCE.hip[,SOURCE2.hip] -DFLAG=VALUE [...]
    python scripts/build_variant.py NAME SOURCE.hip --file PATH   (compile PATH in place of SOURCE.hip)
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from transmvsnet_amd import build as b  # noqa: E402

name, srcs, flags = sys.argv[1], sys.argv[2].split(","), sys.argv[3:]  # SOURCE may be a comma-separated list
paths = {src: os.path.join(b.CSRC, src) for src in srcs}
if "--file" in flags:
    i = flags.index("--file")
    paths[srcs[0]] = os.path.abspath(flags[i + 1])
    flags = flags[:i] + flags[i + 2:]
b.build()
out = os.path.join(b.ROOT, "variants", name)
os.makedirs(out, exist_ok=True)
objs_v = {}
for src, path in paths.items():
    objs_v[src] = os.path.join(out, src.replace(".hip", ".o"))
    subprocess.run([b.HIPCC, *b.CFLAGS, *flags, "-I", b.CSRC, "-c", path, "-o", objs_v[src]], check=True)
objs = [objs_v.get(s, os.path.join(b.OBJ, s.replace(".hip", ".o"))) for s in b.SOURCES]
lib = os.path.join(out, "libtransmvs_hip.so")
subprocess.run([b.HIPCC, "-shared", f"--offload-arch={b.ARCH}", "-fno-gpu-rdc", "-o", lib, *objs], check=True)
print(lib)
