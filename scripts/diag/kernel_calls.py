"""Per-call durations of the kernels matching a substring, from a rocprofv3 rocpd database, grouped
by grid size: python scripts/diag/kernel_calls.py DB SUBSTRING"""
import sqlite3
import sys
from collections import defaultdict

db, pat = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
gcol = next((g for g in ("grid_size", "grid_size_x", "grid_x", "workgroup_count") if g in cols), None)
q = f"select name, {gcol or 0}, (end-start)/1e3 from kernels where name like ?"
by = defaultdict(list)
for name, grid, us in c.execute(q, (f"%{pat}%",)).fetchall():
    by[(name[:60], grid)].append(us)
for (name, grid), v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    v = sorted(v)
    print(f"{name:60s} grid={grid:>9} calls={len(v):4d} median={v[len(v) // 2]:8.1f} us  total={sum(v):9.1f} us")
