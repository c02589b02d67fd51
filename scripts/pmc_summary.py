"""Summarise rocprofv3 --pmc counter CSVs: per kernel name, mean counter values over dispatches.
usage: python scripts/pmc_summary.py dir1/run_counter_collection.csv [dir2/...] [--match conv]"""
import csv
import sys
from collections import defaultdict

args = sys.argv[1:]
match = ""
if "--match" in args:
    i = args.index("--match")
    match = args[i + 1]
    del args[i:i + 2]
files = args
acc = defaultdict(lambda: defaultdict(list))
for f in files:
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if match and match not in name:
            continue
        acc[name[:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, ctrs in acc.items():
    print(name)
    for c, v in sorted(ctrs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
