"""Summarise a rocprofv3 --stats kernel CSV: top kernels by total time."""
import csv
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total GPU kernel time {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {int(r['Calls']):6d} calls "
          f"{float(r['AverageNs']) / 1e3:9.1f} us {float(r['Percentage']):5.1f}%  {r['Name'][:80]}")
