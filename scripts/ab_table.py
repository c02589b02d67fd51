"""Tabulate scripts/gpu/gpu_ab_f32.sh per-layer logs: one row per (layer, mode), one column per variant (ms)."""
import collections
import sys

d = collections.OrderedDict()
vs = []
for line in open(sys.argv[1]):
    t = line.split()
    if len(t) < 6 or t[1] != "x6" and t[1] != "mfma32":
        continue
    v, mode, layer, ms = t[0], t[2], t[4].rstrip(":"), float(t[5])
    if v not in vs:
        vs.append(v)
    d.setdefault((layer, mode), {})[v] = ms
print("layer mode " + " ".join(vs))
for (layer, mode), r in d.items():
    base = r.get(vs[-1])
    print(layer, mode, " ".join(f"{r.get(v, 0):.4f}" for v in vs),
          f"({r.get(vs[0], 0) / base:.3f}x of {vs[-1]})" if base else "")
