"""Print one step's kernel timeline from a rocprofv3 kernel-trace CSV (last complete step)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "fmt_embed_kernel"
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(first)]
seq = rows[idx[-2]:idx[-1]] if len(idx) > 1 else rows
prev = None
tot = 0
agg = {}
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0
    d = (e - s) / 1e3
    tot += d
    agg[r["Kernel_Name"]] = agg.get(r["Kernel_Name"], 0) + d
    print(f"{r['Kernel_Name'][:34]:34s} grid={r['Grid_Size_X']:>9}x{r['Grid_Size_Y']:<3} dur={d:8.1f}us gap={gap:6.1f} "
          f"vgpr={r['VGPR_Count']:>3} lds={r['LDS_Block_Size']}")
    prev = e
span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
print(f"kernel sum {tot:.1f} us, wall span {span:.1f} us")
for k, v in sorted(agg.items(), key=lambda x: -x[1]):
    print(f"  {k[:40]:40s} {v:8.1f} us")
