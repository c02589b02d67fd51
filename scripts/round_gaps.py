"""Idle time per FedAvg round from a rocprofv3 kernel-trace CSV: rounds are cut at the aggregation
kernel (weighted_sum); for each of the last rounds, GPU-busy time vs span and the idle time in
gaps above a threshold (host work between graph replays, graph-submission stalls)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0  # us
cuts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("weighted_sum_kernel")]
for a, b in zip(cuts[-4:-1], cuts[-3:]):
    seg = rows[a + 1:b + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    busy, idle, n_idle, end, big = 0.0, 0.0, 0, t0, []
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        g = (s - end) / 1e3
        if g > thr:
            idle += g
            n_idle += 1
            if g > 100:
                big.append((round(g), r["Kernel_Name"][:40]))
        busy += (e - s) / 1e3
        end = max(end, e)
    span = (end - t0) / 1e3
    print(f"round: {len(seg)} kernels, span {span / 1e3:.2f} ms, busy {busy / 1e3:.2f} ms, "
          f"{n_idle} gaps > {thr:.0f} us = {idle / 1e3:.2f} ms; gaps > 100 us: {big[:12]}")
