"""Aggregate rocprofv3 counter_collection CSVs per kernel name (mean per dispatch)."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for path in glob.glob(f"gpurun_out/{tag}/pmc_*/run_counter_collection.csv"):
    for r in csv.DictReader(open(path)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({c for k in vals.values() for c in k})
print("kernel".ljust(28), " ".join(n[-14:].rjust(14) for n in names))
for k, d in sorted(vals.items()):
    print(k[:28].ljust(28), " ".join(f"{(sum(d[n]) / len(d[n]) if d.get(n) else float('nan')):14.4g}" for n in names))
