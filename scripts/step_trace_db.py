"""One training step's kernels, in launch order, from a rocprofv3 --kernel-trace results database:
duration, idle gap before the kernel (start - latest end so far; negative = overlapping an earlier
kernel, e.g. the side-stream WGRAD), workgroups and name; then the step's kernel count, summed kernel
time, span and union-busy time (the wall time at least one kernel ran).

    python scripts/step_trace_db.py run_results.db
"""
import os
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name,start,end,grid_x*grid_y*grid_z/(workgroup_x*workgroup_y*workgroup_z) from kernels "
                 "order by start").fetchall()
mark = os.environ.get("STEP_MARK", "sgd_")  # the kernel that ends a step (LLaMA: adam_)
idx = [i for i, r in enumerate(rows) if r[0].startswith(mark)]
a, b = idx[-3], idx[-2]
tot = 0.0
busy = 0.0
last_end = rows[a][2]
gaps = 0.0
for r in rows[a + 1:b + 1]:
    d = (r[2] - r[1]) / 1e3
    tot += d
    gap = (r[1] - last_end) / 1e3
    if gap > 0:
        gaps += gap
        busy += d
    else:
        busy += max(0.0, (r[2] - last_end) / 1e3)
    last_end = max(last_end, r[2])
    print(f"{d:8.1f} us gap {gap:7.1f} wgs {r[3]:6d} {r[0][:60]}")
span = (rows[b][2] - rows[a][2]) / 1e3
print("kernels", b - a, "sum", round(tot, 1), "span", round(span, 1), "busy", round(busy, 1),
      f"({100 * busy / span:.1f} %)", "idle gaps", round(gaps, 1))
