"""Per-kernel-name totals of two one-step traces (scripts/step_trace_db.py output): A vs B."""
import re
import sys
from collections import defaultdict


def load(path):
    tot, cnt = defaultdict(float), defaultdict(int)
    for ln in open(path):
        m = re.match(r"\s*([\d.]+) us wgs\s+\d+ (.*)", ln)
        if not m:
            continue
        name = re.sub(r"^void ", "", m.group(2)).split("(")[0]
        name = re.sub(r"\(anonymous namespace\)::", "", name)
        tot[name] += float(m.group(1))
        cnt[name] += 1
    return tot, cnt


a, ca = load(sys.argv[1])
b, cb = load(sys.argv[2])
print(f"{'A us':>9} {'n':>3} {'B us':>9} {'n':>3} {'B-A':>8}  kernel")
for k in sorted(set(a) | set(b), key=lambda k: -(a.get(k, 0) + b.get(k, 0))):
    print(f"{a.get(k, 0):9.1f} {ca.get(k, 0):3d} {b.get(k, 0):9.1f} {cb.get(k, 0):3d} {b.get(k, 0) - a.get(k, 0):8.1f}  {k}")
print(f"{sum(a.values()):9.1f} {sum(ca.values()):3d} {sum(b.values()):9.1f} {sum(cb.values()):3d}  total")
