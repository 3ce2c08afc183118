"""Every counter's mean per (kernel, grid) from scripts/pmc_kernel.sh passes, raw (no derived ratios).

    python scripts/diag/pmc_dump.py TAG [name-filter]
"""
import collections
import csv
import glob
import re
import sys

tag = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sorted(glob.glob(f"gpurun_out/{tag}/pmc_*/run_counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        name = re.sub(r"^void tmvs::|\(.*$", "", r["Kernel_Name"])[:70]
        if filt and filt not in name:
            continue
        vals[(name, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (name, grid), d in sorted(vals.items()):
    print(f"{name} grid={grid}")
    for k in sorted(d):
        print(f"    {k:40s} {sum(d[k]) / len(d[k]):16.1f}")
