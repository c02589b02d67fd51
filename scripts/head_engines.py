"""fp32 LM-head products (T x 288 -> 32000) on the two native engines: the conv engine (1x1 conv over
T pixels, fp32 operands) vs the X6 planes GEMM (pre-split planes), plus the plane splits.

    python scripts/head_engines.py [--T 8192]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.ops import functional as Fn  # noqa: E402
from ddl25spring_amd.ops import gemm_x6 as G  # noqa: E402


def timeit(fn, iters=10, warm=2):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8192)
    ap.add_argument("--plans", default="4,4,3,1;3,4,3,1;4,4,3,2;4,2,4,1")
    args = ap.parse_args()
    dev = torch.device("cuda")
    T, C, K = args.T, 288, 32000
    x = torch.randn(T, C, device=dev)
    w = torch.randn(K, C, device=dev) * 0.05
    dy = torch.randn(T, K, device=dev) * 0.01
    geom = Fn.ConvGeom(1, T, 1, 1, C, K, 1, 1, 1, 0)
    x5, w5, d5 = x.view(1, T, 1, 1, C), w.view(1, K, 1, 1, C), dy.view(1, T, 1, 1, K)
    dwt = torch.zeros(1, K, 1, 1, C, device=dev)
    res = {"conv_us": {"fwd": timeit(lambda: Fn.conv_fwd(x5, w5, geom)),
                       "dgrad": timeit(lambda: Fn.conv_dgrad(d5, w5, geom)),
                       "wgrad": timeit(lambda: Fn.conv_wgrad(d5, x5, geom, dwt))}}
    px, pw, pd = G.split(x), G.split(w), G.split(dy)
    res["split_us"] = {"x": timeit(lambda: G.split(x, px.data)), "w": timeit(lambda: G.split(w, pw.data)),
                       "dy": timeit(lambda: G.split(dy, pd.data))}
    prods = {"fwd": (pw, False, px, False, (T, K), C), "dgrad": (pw, True, pd, False, (T, C), K),
             "wgrad": (px, True, pd, True, (K, C), T)}
    x6 = {}
    for mode, (pa, amn, pb, bmn, oshape, Kr) in prods.items():
        out = torch.zeros(*oshape, device=dev)
        M, N = oshape[1], oshape[0]
        best = None
        for pl in args.plans.split(";"):
            p = tuple(int(v) for v in pl.split(","))
            G._PLANS.clear()
            G._PLANS[(M, N, Kr)] = p
            t = timeit(lambda: G.gemm(pa, amn, pb, bmn, out, accumulate=mode == "wgrad"))
            if best is None or t < best[0]:
                best = (t, p)
        G._PLANS.clear()
        x6[mode] = {"us": best[0], "plan": best[1]}
    res["x6g"] = x6
    print(json.dumps(res))


if __name__ == "__main__":
    main()
