"""Average duration per (kernel, grid) from a rocprofv3 rocpd database, optionally filtered by a substring.

    python scripts/diag/kernel_grid_times.py run_results.db [substring ...]
"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
pats = sys.argv[2:] or [""]
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
grid = [x for x in cols if "grid" in x.lower()][0]
where = " or ".join("name like ?" for _ in pats)
q = f"select name, {grid}, count(*), avg(end-start)/1e3 from kernels where {where} group by name, {grid} order by 4 desc"
for name, g, n, us in c.execute(q, [f"%{p}%" for p in pats]):
    print(f"{us:9.1f} us  x{n:4d}  grid={g:9d}  {name[:90]}")
