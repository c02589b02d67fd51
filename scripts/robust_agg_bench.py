"""Robust aggregation time at world 1 (fl/aggregate.py): median / trimmed mean / Krum / mean over
K client updates of P floats (default 8 x 11.2M, ResNet-18's size), CUDA-event timed.

    python scripts/robust_agg_bench.py [--K 8] [--P 11173962] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.fl import aggregate as A  # noqa: E402
from ddl25spring_amd.runtime.dist import DistContext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=8)
    ap.add_argument("--P", type=int, default=11_173_962)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda")
    ctx = DistContext(device=dev)
    rows = torch.randn(args.K, args.P, device=dev) * 0.01
    coeffs = torch.full((args.K,), 1.0 / args.K, device=dev)
    out = torch.empty(args.P, device=dev)
    res = {"K": args.K, "P": args.P}
    for name in ("mean", "median", "trimmed_mean", "krum"):
        agg = A.make_aggregator(name, trim=0.25, f=2)
        call = (lambda: agg(ctx, rows, coeffs, out)) if name == "mean" else (lambda: agg(ctx, rows, [args.K], args.P))
        for _ in range(3):
            call()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(args.iters):
            call()
        e.record()
        torch.cuda.synchronize()
        res[name + "_ms"] = round(s.elapsed_time(e) / args.iters, 3)
    res["hbm_read_once_ms"] = round(args.K * args.P * 4 / 5.0e12 * 1e3, 3)  # at 5 TB/s achievable
    print(json.dumps(res))


if __name__ == "__main__":
    main()
