"""Per-(kernel, grid) mean duration (us) and per-step total from a rocprofv3 kernel trace CSV."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
# steady state only: drop the setup dispatches (weight uploads, packing) before the first forward step
first = next((i for i, r in enumerate(rows) if "fmt_embed" in r["Kernel_Name"]), 0)
rows = rows[first:]
steps = max(1, sum(1 for r in rows if r["Kernel_Name"].startswith("fmt_embed") or "fmt_embed" in r["Kernel_Name"]))
agg = collections.defaultdict(list)
for r in rows:
    name = re.sub(r"^void tmvs::|\(.*$", "", r["Kernel_Name"])
    name = re.sub(r"^tmvs::", "", name)[:70]
    agg[(name, r.get("Grid_Size", r.get("Grid_Size_X", "?")))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
out = []
for (name, grid), v in agg.items():
    # median per call x calls per step: one cold call (first touch of a fresh allocation in a
    # warm-up step, e.g. 25 ms for a 255-MB conv0 output) must not stand in for the steady state
    med = sorted(v)[len(v) // 2]
    per_step = med * len(v) / steps
    tot += per_step
    out.append((per_step, name, grid, len(v) / steps, med))
for per_step, name, grid, calls, mean in sorted(out, reverse=True):
    print(f"{per_step:9.1f} us/step  {calls:4.1f} calls x {mean:8.1f} us  grid={grid:>9}  {name}")
print(f"{tot:9.1f} us/step total over {steps} steps (median duration per call)")
