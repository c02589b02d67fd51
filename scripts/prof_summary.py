"""Per-kernel time summary of a rocprofv3 --kernel-trace results database (rocpd sqlite).

    python scripts/prof_summary.py gpurun_out/prof/run_results.db [--top 40] > profiles/x.txt
"""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=40)
a = ap.parse_args()
cur = sqlite3.connect(a.db).cursor()
tot = cur.execute("select sum(end-start)/1e6 from kernels").fetchone()[0]
span = cur.execute("select (max(end)-min(start))/1e6 from kernels").fetchone()[0]
print(f"kernels: {tot:.1f} ms of GPU time over a {span:.1f} ms span")
print(f"{'total ms':>10} {'share':>6} {'calls':>7} {'avg us':>9}  kernel")
for n, c, s, av in cur.execute("select name, count(*), sum(end-start)/1e6, avg(end-start)/1e3 from kernels "
                               "group by name order by sum(end-start) desc limit ?", (a.top,)):
    print(f"{s:10.1f} {100 * s / tot:5.1f}% {c:7d} {av:9.1f}  {n[:120]}")
