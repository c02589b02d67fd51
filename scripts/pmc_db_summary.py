"""Per-kernel mean PMC values from rocprofv3 SQLite DBs (counters_collection view).
usage: python scripts/pmc_db_summary.py run1.db [run2.db ...] [--match conv_igemm]"""
import sqlite3
import sys
from collections import defaultdict

args = sys.argv[1:]
match = ""
if "--match" in args:
    i = args.index("--match")
    match = args[i + 1]
    del args[i:i + 2]
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for db in args:
    c = sqlite3.connect(db)
    for name, ctr, val, d, disp in c.execute(
            "select kernel_name, counter_name, value, duration, dispatch_id from counters_collection"):
        if match and match not in name:
            continue
        acc[name[:60]][ctr].append(val)
        dur[name[:60]].append((disp, d))
for name, ctrs in acc.items():
    ds = dict(dur[name])
    print(f"{name}  (dispatches {len(ds)}, mean {sum(ds.values()) / max(1, len(ds)) / 1e3:.1f} us)")
    for k, v in sorted(ctrs.items()):
        print(f"   {k:30s} {sum(v) / len(v):16.1f}")
