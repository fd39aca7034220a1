"""Per-kernel summary of a rocprofv3 SQLite output (run_results.db): calls, mean /
total time, grid, VGPRs, LDS, scratch.  usage: python tools/prof_db.py <db> [N]"""
import sqlite3
import sys

db = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(duration)/1000.0, sum(duration)/1e6, max(grid_x), "
                 "max(workgroup_x), max(vgpr_count), max(lds_size), max(scratch_size) from kernels "
                 "group by name order by sum(duration) desc limit ?", (n,)).fetchall()
print("| kernel | calls | mean us | total ms | grid | wg | VGPR | LDS B | scratch |")
print("|---|---|---|---|---|---|---|---|---|")
for r in rows:
    name = r[0].replace("void ", "").replace("(anonymous namespace)::", "")[:60]
    print(f"| `{name}` | {r[1]} | {r[2]:.2f} | {r[3]:.2f} | {r[4]} | {r[5]} | {r[6]} | {r[7]} | {r[8]} |")
