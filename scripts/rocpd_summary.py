"""Per-kernel statistics from a rocprofv3 SQLite (rocpd) database -> kernel_stats-style CSV + text.

usage: python scripts/rocpd_summary.py results.db out_prefix [top]
Writes <out_prefix>_kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs, VGPR, AGPR, LDS, Grid, Block) and prints the top kernels.
"""
import csv
import sqlite3
import sys

db, prefix = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
c = sqlite3.connect(db)
rows = c.execute(
    "select name, count(*), sum(duration), min(duration), max(duration), max(vgpr_count), "
    "max(accum_vgpr_count), max(lds_size), max(grid_x*grid_y*grid_z), max(workgroup_x*workgroup_y*workgroup_z) "
    "from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows)
span = c.execute("select min(start), max(end) from kernels").fetchone()
with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                "VGPR", "AGPR", "LDS", "GridThreads", "Block"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], r[2] / r[1], 100.0 * r[2] / tot, r[3], r[4], r[5], r[6], r[7], r[8], r[9]])
print(f"total GPU kernel time {tot / 1e6:.2f} ms over {sum(r[1] for r in rows)} dispatches; "
      f"trace span {(span[1] - span[0]) / 1e6:.2f} ms")
for r in rows[:top]:
    print(f"{r[2] / 1e6:9.2f} ms {r[1]:6d} calls {r[2] / r[1] / 1e3:9.1f} us {100 * r[2] / tot:5.1f}% "
          f"vgpr {r[5]:3d} lds {r[7]:6d}  {r[0][:90]}")
