"""Compact per-kernel VGPR/SGPR/spill/occupancy table (hipcc -Rpass-analysis=kernel-resource-usage)."""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-I", "include",
       "-c", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: +([A-Za-z ]+\[?[a-zA-Z/]*\]?): (\S+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if filt and filt not in k:
        continue
    print(f"{k[:90]:90s} vgpr={v.get('VGPRs','?'):>4} agpr={v.get('AGPRs','?'):>3} sgpr={v.get('SGPRs','?'):>4} "
          f"vspill={v.get('VGPRs Spill','?'):>4} sspill={v.get('SGPRs Spill','?'):>5} occ={v.get('Occupancy [waves/SIMD]','?')} "
          f"lds={v.get('LDS Size [bytes/block]','?')}")
