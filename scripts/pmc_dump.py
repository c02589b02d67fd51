"""Mean of every collected counter per matching kernel over all rocprofv3 --pmc passes under a dir.
usage: python scripts/pmc_dump.py <dir> [kernel-name-substring]"""
import glob
import sqlite3
import sys
from collections import defaultdict

root, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
acc = defaultdict(lambda: defaultdict(list))
for db in glob.glob(f"{root}/**/*.db", recursive=True):
    c = sqlite3.connect(db)
    for name, ctr, val in c.execute("select kernel_name, counter_name, value from counters_collection"):
        if pat in name:
            acc[name.split("(")[0].replace("void ", "")][ctr].append(val)
for k, d in acc.items():
    print(f"== {k}")
    for ctr in sorted(d):
        v = d[ctr]
        print(f"  {ctr:40s} {sum(v) / len(v):16.1f}  (n={len(v)})")
