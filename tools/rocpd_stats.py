"""Per-kernel stats (count, mean / min us) from a rocprofv3 rocpd SQLite file.

  python tools/rocpd_stats.py gpurun_out/prof/.../run_results.db [name-filter]
"""
import sqlite3
import sys

db = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, count(*), avg(end - start), min(end - start) from kernels "
                 f"group by {name} order by sum(end - start) desc").fetchall()
print(f"{'count':>6} {'mean_us':>9} {'min_us':>9}  kernel")
for n, cnt, avg, mn in rows:
    if flt in n:
        print(f"{cnt:6d} {avg / 1e3:9.2f} {mn / 1e3:9.2f}  {n[:150]}")
