"""Print a rocprofv3 kernel_stats.csv sorted by total time (name truncated). Usage: stats_table.py CSV [N]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:9.1f} us "
          f"{100*float(r['TotalDurationNs'])/tot:5.1f}%  {r['Name'][:110]}")
print(f"total {tot/1e6:.3f} ms")
