"""X6 GEMM (csrc/kernels/gemm_x6.hip) on the fp32 LLaMA's linear products vs the vendor fp32 GEMM
(torch.mm -> hipBLASLt): time per product and error against float64.

    python scripts/gemm_x6_bench.py [--T 8192] [--plans "4,4,4,1;3,4,4,2"] [--check]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from ddl25spring_amd.ops import gemm_x6 as G  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8192)
    ap.add_argument("--plans", default="", help="';'-separated TP,TQ,NS,split to try per product")
    ap.add_argument("--check", action="store_true", help="float64 error check")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    T = args.T
    shapes = [("qkv", 288, 864), ("wo", 288, 288), ("w13", 288, 1536), ("w2", 768, 288), ("head", 288, 32000)]
    for name, Kin, Nout in shapes:
        if args.only and name not in args.only.split(","):
            continue
        x = torch.randn(T, Kin, device=dev)
        w = torch.randn(Nout, Kin, device=dev) * 0.05
        dy = torch.randn(T, Nout, device=dev) * 0.01
        px, pw, pd = G.split(x), G.split(w), G.split(dy)
        assert torch.equal(px.dense(), x) and torch.equal(pw.dense(), w), "planes not exact"
        t_split = timeit(lambda: G.split(dy, pd.data))
        prods = {
            "fwd": (lambda o, **k: G.gemm(pw, False, px, False, o, **k), (T, Nout), lambda: x @ w.t(),
                    lambda: x.double() @ w.double().t(), 2 * T * Kin * Nout),
            "dgrad": (lambda o, **k: G.gemm(pw, True, pd, False, o, **k), (T, Kin), lambda: dy @ w,
                      lambda: dy.double() @ w.double(), 2 * T * Kin * Nout),
            "wgrad": (lambda o, **k: G.gemm(px, True, pd, True, o, **k), (Nout, Kin), lambda: dy.t() @ x,
                      lambda: dy.double().t() @ x.double(), 2 * T * Kin * Nout),
        }
        for mode, (ours, oshape, vend, ref64, flop) in prods.items():
            out = torch.empty(*oshape, device=dev)
            M, N = oshape[1], oshape[0]
            K = {"fwd": Kin, "dgrad": Nout, "wgrad": T}[mode]
            rows = []
            plans = [None] + ([tuple(int(v) for v in p.split(",")) for p in args.plans.split(";")] if args.plans else [])
            for pl in plans:
                G._PLANS.clear()
                if pl is not None:
                    G._PLANS[(M, N, K)] = pl
                used = G.plan(M, N, K)
                t_ours = timeit(lambda: ours(out))
                rec = {"prod": name, "mode": mode, "M": M, "N": N, "K": K, "plan": used, "us": round(t_ours, 1),
                       "tflops": round(flop / t_ours / 1e6, 1)}
                if args.check:
                    ours(out)
                    r = ref64()
                    v = vend().double()
                    scale = r.abs().max().item()
                    rec["err"] = (out.double() - r).abs().max().item() / scale
                    rec["vendor_err"] = (v - r).abs().max().item() / scale
                rows.append(rec)
            t_v = timeit(vend)
            for rec in rows:
                rec["vendor_us"] = round(t_v, 1)
                rec["split_us"] = round(t_split, 1)
                print(json.dumps(rec), flush=True)
    G._PLANS.clear()


if __name__ == "__main__":
    main()
