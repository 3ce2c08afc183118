"""Print one step's kernel timeline (start offset, duration) from a rocprofv3 kernel trace CSV."""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "fmt_embed" in r["Kernel_Name"]]
k = starts[-2] if len(starts) > 1 else starts[0]
end = starts[-1] if len(starts) > 1 else len(rows)
t0 = int(rows[k]["Start_Timestamp"])
for r in rows[k:end]:
    name = re.sub(r"^void |^tmvs::|\(.*$|<.*$", "", r["Kernel_Name"]).replace("tmvs::", "")[:40]
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q={r.get('Queue_Id', r.get('Stream_Id', '?')):>3}  {name}")
