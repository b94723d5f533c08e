"""Per-kernel duration summary from a rocprofv3 SQLite output (rocpd 'kernels' view)."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = db.execute(f"select {name_col}, count(*), avg(end - start), sum(end - start) from kernels group by {name_col} order by sum(end - start) desc").fetchall()
print("Name,Calls,AverageNs,TotalDurationNs")
for n, cnt, avg, tot in rows:
    print(f'"{n}",{cnt},{avg:.1f},{tot}')
