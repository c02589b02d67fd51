"""Communication / compute overlap in a rocprofv3 --kernel-trace database: for every collective
kernel (RCCL all-reduce etc.), the fraction of its duration during which a non-collective kernel
ran too, and which compute kernels it overlapped.

    python scripts/overlap_report.py gpurun_out/r50_prof/run_results.db > profiles/x.txt
"""
import argparse
import sqlite3
from collections import Counter

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--pattern", default="nccl,rccl,AllReduce,allreduce")
a = ap.parse_args()
pats = [p.lower() for p in a.pattern.split(",")]
cur = sqlite3.connect(a.db).cursor()
rows = cur.execute("select name, start, end from kernels order by start").fetchall()
comm = [(n, s, e) for n, s, e in rows if any(p in n.lower() for p in pats)]
comp = [(n, s, e) for n, s, e in rows if not any(p in n.lower() for p in pats)]
print(f"{len(rows)} kernels, {len(comm)} collective kernels")
tot_c = sum(e - s for _, s, e in comm)
tot_ov = 0
names = Counter()
for n, s, e in comm:
    iv = sorted((max(s, cs), min(e, ce), cn) for cn, cs, ce in comp if cs < e and ce > s)
    cov, cur_end = 0, s
    for lo, hi, cn in iv:
        names[cn[:80]] += 1
        lo = max(lo, cur_end)
        if hi > lo:
            cov += hi - lo
            cur_end = hi
    tot_ov += cov
    print(f"{(e - s) / 1e3:9.1f} us  overlapped {100 * cov / max(1, e - s):5.1f}%  {n[:90]}")
if comm:
    print(f"collective kernel time {tot_c / 1e6:.3f} ms, {100 * tot_ov / max(1, tot_c):.1f}% of it concurrent "
          "with compute kernels")
    print("compute kernels seen running during collectives:")
    for n, c in names.most_common(15):
        print(f"  {c:5d}  {n}")
