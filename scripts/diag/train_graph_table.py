"""Split a rocprofv3 kernel trace at host gaps > 20 ms and table the last segment's kernels by total time.
    python scripts/diag/train_graph_table.py run_kernel_trace.csv [N]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
segs, cur, last_end = [], [], None
for r in rows:
    s = int(r["Start_Timestamp"])
    if last_end is not None and s - last_end > 20e6:
        segs.append(cur)
        cur = []
    cur.append(r)
    last_end = max(last_end or 0, int(r["End_Timestamp"]))
segs.append(cur)
seg = segs[-1]
wall = (max(int(r["End_Timestamp"]) for r in seg) - int(seg[0]["Start_Timestamp"])) / 1e6
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    name = re.sub(r"\(.*$", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "").replace("tmvs::", "")
    agg[name][0] += 1
    agg[name][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"segments {len(segs)}; last: {len(seg)} kernels, wall {wall:.2f} ms, kernel sum {tot / 1e3:.2f} ms")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:n]:
    print(f"{t:9.1f} us {c:5d} x {t / c:8.1f}  {k[:110]}")
