"""Per-kernel totals from a rocprofv3 rocpd database (kernels view): name, calls, total ms, ms/step."""
import sqlite3
import sys

db, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(end-start)/1e6 from kernels group by name order by 3 desc").fetchall()
print(f"total {sum(r[2] for r in rows):.2f} ms over {steps} steps")
for name, n, ms in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{ms / steps:9.3f} ms/step {n:6d} calls  {name[:100]}")
