"""Per-phase clock of the one-launch split-NN epoch (csrc/kernels/mlp_epoch.hip, the phase clock
of MlpEpoch.prof): us per mini-batch for every forward / backward level, the CE and AdamW, plus
the whole epoch's time by CUDA events. Heart split-NN shapes (2 parties x 15 features, 821 rows,
batch 64), random data.

    python scripts/mlp_epoch_prof.py [--epochs 20] [--batch 64]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.models import tabular as T  # noqa: E402
from ddl25spring_amd.ops import mlp_epoch as ME  # noqa: E402
from ddl25spring_amd.optim import FlatAdamW  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--n", type=int, default=821)
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    bottoms = [T.BottomModel(15, 30).to(dev) for _ in range(2)]
    top = T.TopModel(bottoms, 2).to(dev)
    opt = FlatAdamW([*[p for b in bottoms for p in b.parameters()], *top.parameters()])
    eng = ME.MlpEpoch(ME.splitnn_graph(bottoms, top), opt, args.batch, seed=1)
    xs = [torch.randn(args.n, 15, device=dev) for _ in range(2)]
    y = torch.nn.functional.one_hot(torch.randint(0, 2, (args.n,), device=dev), 2).float()
    stats = torch.zeros(2, device=dev)
    for _ in range(3):
        eng.run(xs, y, stats)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(args.epochs):
        eng.run(xs, y, stats)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / args.epochs
    eng.prof = torch.zeros(ME.NPROF, dtype=torch.int64, device=dev)
    for _ in range(args.epochs):
        eng.run(xs, y, stats)
    torch.cuda.synchronize()
    steps = args.epochs * -(-args.n // args.batch)
    ticks = eng.prof.cpu().tolist()
    g = eng.g
    names = {lv: f"fwd{lv}" for lv in range(g.nlev)}
    names[ME.MAXLEV] = "ce"
    names.update({ME.MAXLEV + 1 + lv: f"bwd{lv}" for lv in range(g.nlev)})
    names[ME.NPROF - 1] = "adamw"
    per = {names[i]: round(t * 10e-3 / steps, 2) for i, t in enumerate(ticks) if i in names}  # 100 MHz ticks -> us
    print(json.dumps({"ms_per_epoch": round(ms, 3), "samples_per_s": round(args.n / ms * 1e3, 1),
                      "us_per_step": round(ms * 1e3 / -(-args.n // args.batch), 1), "phase_us_per_step": per}))


if __name__ == "__main__":
    main()
